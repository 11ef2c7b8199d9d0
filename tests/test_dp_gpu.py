"""Data-parallel train step on the GPU, two ranks (tools/dp_check.py under torch.distributed.run).
On a one-GPU box both ranks share device 0 and gloo carries the collectives (RCCL refuses two
ranks on one GPU); the engine's bucketed, hook-driven all-reduce and its deferred weight
gradients are the same code the RCCL run uses.  The step must equal the shard-weighted average
of single-process steps, and every rank must end it with bitwise identical gradients and weights."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("global_batch,deferred", [(4, False), (5, False), (5, True)])
def test_dp_two_ranks_equal_weighted_single_process(global_batch, deferred):
    """tools/dp_check.py: the DP step equals sum_r (n_r / n) x (single-process gradient of shard r)
    through AdamW (equal shards 2+2 and unequal 3+2), and the ranks agree bitwise.  deferred: the
    64-output blocks' weight gradients go to the deferred side-stream pass, so the bucketed
    all-reduce's low-water reports wait for a pending deferral."""
    env = dict(os.environ)
    env["DP_CHECK_GLOBAL"] = str(global_batch)
    env["DP_CHECK_DEFERRED"] = "1" if deferred else "0"
    if torch.cuda.device_count() < 2:
        env["UNET_DP_ONE_DEVICE"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "dp_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "identical across ranks: True" in r.stdout
    assert r.stdout.count("equal to expected: True") == 2, r.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("global_batch,drop", [(4, False), (5, False), (5, True)])
def test_dp_sync_bn_equals_full_batch(global_batch, drop):
    """tools/dp_syncbn_check.py: with SyncBN (model.enable_data_parallel(sync_bn=True), SURVEY 8(e)
    option) a two-rank step over shards 2+2 / 3+2 equals ONE single-process step over the whole
    global batch (dropout off): gradients within fp32 reduction order, moving statistics equal,
    and every rank bitwise identical.  drop: dropout 0.2 with SyncBN, against the same DP step
    through the unfused BN-backward statistics route (the dropout-masked producer
    partials feeding the SyncBN all-reduce)."""
    env = dict(os.environ)
    env["DP_CHECK_GLOBAL"] = str(global_batch)
    env["DP_CHECK_DROP"] = "1" if drop else "0"
    if torch.cuda.device_count() < 2:
        env["UNET_DP_ONE_DEVICE"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tools", "dp_syncbn_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "identical across ranks: True" in r.stdout
    assert r.stdout.count("equal to full batch: True") == 2, r.stdout[-2000:]


@pytest.mark.gpu
def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` (the driver's command shape, no launcher environment) runs two
    ranks: the parent starts torch.distributed.run as a child before touching the GPU, and the
    JSON line reports both GPUs and the global batch."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if torch.cuda.device_count() < 2:
        env["UNET_DP_ONE_DEVICE"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-roofline", "--encoder-batch", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 32, out
    assert out["config"]["parallelism"] == "dp2"
    dp = out["data_parallel"]  # the all-reduce exposure pass
    assert dp["backend"] in ("nccl", "gloo") and dp["buckets"] >= 1 and dp["allreduce_exposed_ms"] >= 0
    assert sum(dp["bucket_bytes"]) == dp["grad_bytes"]
    if torch.cuda.device_count() >= 2:
        assert dp["backend"] == "nccl"  # RCCL
