"""bench.py's JSON line on the host (no GPU): the contract fields the driver reads, and the
data-parallel object under WORLD_SIZE=8 with a mocked process group, so the first 8-GPU node the
driver gets produces a complete line (reference: single process,
/root/reference/scripts/train.py:119-130)."""
import argparse

import pytest
import torch

import bench
from unet_amd import dp
from unet_amd.params import count_params, flat_layout, unet_variables

GRAD_NUMEL = flat_layout(unet_variables(3, 1), True).total  # the flat gradient buffer (padded slices)


def _args(*argv):
    return bench.parse_args(list(argv))


def test_single_gpu_line_contract():
    a = _args()
    assert (a.gpus, a.steps, a.warmup, a.batch, a.size, a.num_classes) == (1, 20, 5, 16, 256, 1)
    out = bench.result_line(a, 1, 0.2, 0.5)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["value"] == pytest.approx(16 * 20 / 0.2)
    assert out["ms_per_step"] == pytest.approx(10.0) and out["scaling"] == "weak"
    assert out["config"]["workload"].startswith("configs[1]") and out["config"]["parallelism"] == "dp1"


class _FakeDist:
    """The slice of torch.distributed GradBucketer uses, for a world of 8 (no rendezvous)."""

    ReduceOp = torch.distributed.ReduceOp

    def __init__(self, world):
        self.world, self.calls = world, []

    def is_initialized(self):
        return True

    def get_world_size(self, group=None):
        return self.world

    def all_reduce(self, t, op=None, group=None, async_op=False):
        self.calls.append((t.data_ptr(), t.numel()))

        class _W:
            def wait(self):
                return None
        return _W()


def test_world8_line_has_data_parallel_fields(monkeypatch):
    fake = _FakeDist(8)
    monkeypatch.setattr(dp, "dist", fake)
    monkeypatch.setenv("WORLD_SIZE", "8")
    grads = torch.zeros(GRAD_NUMEL)
    bk = dp.GradBucketer(grads)  # the engine's default 6 MB buckets
    assert bk.world == 8
    # the backward reports low-water marks head -> enc1; every bucket goes out exactly once
    for lw in range(GRAD_NUMEL, -1, -GRAD_NUMEL // 7):
        bk.ready(max(lw, 0))
    assert bk.finish() == pytest.approx(1 / 8)
    assert sum(n for _, n in fake.calls) == GRAD_NUMEL and len(fake.calls) == len(bk.buckets) == 4
    a = _args("--gpus", "8")
    out = bench.result_line(a, 8, 0.2, 0.5)
    out["data_parallel"] = bench.dp_info_obj("nccl", 0.05, bk, a.steps)
    assert out["n_gpus"] == 8 and out["config"]["global_batch"] == 128 and out["config"]["parallelism"] == "dp8"
    assert out["value"] == pytest.approx(8 * 16 * 20 / 0.2)
    d = out["data_parallel"]
    assert d["backend"] == "nccl" and d["world"] == 8 and d["buckets"] == 4
    assert sum(d["bucket_bytes"]) == d["grad_bytes"] == 4 * GRAD_NUMEL
    assert count_params(unet_variables(3, 1))[0] * 4 <= d["grad_bytes"] < 24.1e6  # 23.95 MB of gradients
    assert d["ring_bytes_per_gpu"] == round(2 * 7 / 8 * d["grad_bytes"])  # 41.9 MB
    assert d["allreduce_exposed_ms"] == 0.05


def test_world_mismatch_is_refused(monkeypatch):
    """--gpus N under a launcher that started a different number of ranks is an error (main())."""
    a = _args("--gpus", "4")
    assert a.gpus == 4
    with pytest.raises(SystemExit):
        bench.parse_args(["--gpus", "0"])
    assert isinstance(a, argparse.Namespace)
