"""Data-parallel plumbing on CPU with the gloo backend (world size 2, 4 and 8): the same
GradBucketer the GPU path uses (RCCL there) averages a flat gradient buffer exactly, with
buckets launched as the backward's low-water mark passes them; sharding of a global batch;
and DP with the oracle as each rank's compute equals the single-process average."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from unet_amd.dp import GradBucketer, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 10007
        g = torch.arange(n, dtype=torch.float32) * (rank + 1)
        b = GradBucketer(g, bucket_bytes=4 * 1000)
        assert len(b.buckets) == 11
        # simulate backward: low-water mark decreasing from the end of the buffer
        for lw in range(n, -1, -997):
            b.ready(max(lw, 0))
        scale = b.finish()
        ref = torch.arange(n, dtype=torch.float32) * sum(range(1, world + 1))
        ok1 = torch.equal(g, ref) and abs(scale - 1.0 / world) < 1e-12
        # oracle-as-compute DP with UNEQUAL shards (5 images: 3+2 over 2 ranks, 2+1+1+1 over 4):
        # each rank's gradient of its shard-mean dice loss, weighted n_local * world / n_global
        # (the head backward's loss_scale), summed by the all-reduce and scaled 1/world (AdamW's
        # grad_scale), must be the gradient of the global-batch mean loss
        from oracle import keras_ops as K
        G = 5
        rng = np.random.default_rng(0)
        yt = (rng.random((G, 8, 8, 1)) > 0.5).astype(np.float64)
        yp = rng.random((G, 8, 8, 1))
        lo, hi = shard_bounds(G, world, rank)
        loss_scale = (hi - lo) * world / G
        gl = torch.from_numpy(loss_scale * K.dice_loss_grad(yt[lo:hi], yp[lo:hi]))
        full = torch.zeros((G, 8, 8, 1), dtype=torch.float64)
        full[lo:hi] = gl
        dist.all_reduce(full)
        ref2 = K.dice_loss_grad(yt, yp)
        ok2 = np.allclose(full.numpy() / world, ref2, rtol=1e-12, atol=1e-15)
        q.put((rank, ok1, ok2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])  # 8: the driver's scaling node, rehearsed on CPU
def test_bucketed_allreduce_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok1 and ok2 for _, ok1, ok2 in res), res


def test_shard_bounds():
    assert [shard_bounds(128, 8, r) for r in (0, 7)] == [(0, 16), (112, 128)]
    assert [shard_bounds(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    with pytest.raises(ValueError):
        shard_bounds(8, 2, 2)


def test_single_process_is_noop():
    g = torch.ones(100)
    b = GradBucketer(g)
    b.ready(0)
    assert b.finish() == 1.0 and torch.equal(g, torch.ones(100))
