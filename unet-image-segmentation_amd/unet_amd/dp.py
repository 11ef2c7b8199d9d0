"""Data parallelism: one process per GPU, the minibatch sharded across ranks, one gradient
all-reduce per step (RCCL over xGMI via torch.distributed backend "nccl").

The reference has no distribution (single process, scripts/train.py:119-130 only enables
memory growth).  Design for MI355X:
  * the 82 gradient tensors are one flat buffer (params.py), cut into a few contiguous
    buckets (~6 MB by default: 4 buckets for 24 MB);
  * backward produces gradients from the head down to enc1, i.e. from the END of the flat
    buffer to its start; the engine reports a low-water offset after every layer and a
    bucket is all-reduced (async, on RCCL's stream) as soon as it is complete, so the
    collectives overlap the remaining backward kernels;
  * the average (x 1/world) is folded into the AdamW kernel's grad_scale: no extra pass; a
    rank whose shard is not 1/world of the global batch weights its loss gradient by
    n_local * world / n_global (head backward's loss_scale), so the result is the gradient of
    the global-batch mean for any split;
  * BatchNorm batch statistics are per replica (the tf.distribute default, synchronized=False);
    the moving statistics are averaged over ranks before validation / checkpoints
    (model.sync_bn_statistics; tf.distribute reads them as a MEAN over replicas).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of this rank's shard of a global batch (equal shards; remainder to low ranks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).
    Returns (rank, world, local_rank); (0, 1, 0) without a launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("UNET_DP_ONE_DEVICE") == "1":
        # rehearsal of the multi-rank path on a one-GPU box: every rank on device 0, gloo
        # collectives (RCCL refuses two ranks on one GPU)
        local = 0
        backend = backend or "gloo"
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local


def average_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean of a tensor over the ranks (sum all-reduce, then x 1/world)."""
    if dist.is_initialized():
        world = dist.get_world_size(group)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            t.mul_(1.0 / world)
    return t


class GradBucketer:
    """Bucketed, overlapped all-reduce of a flat gradient buffer."""

    def __init__(self, grads: torch.Tensor, bucket_bytes: int = 6 << 20, group=None):
        self.grads = grads
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        n = grads.numel()
        per = max(1, bucket_bytes // grads.element_size())
        # buckets as [lo, hi) ranges, highest offsets first (they become ready first)
        self.buckets: List[Tuple[int, int]] = []
        hi = n
        while hi > 0:
            lo = max(0, hi - per)
            self.buckets.append((lo, hi))
            hi = lo
        self._next = 0
        self._works = []

    def reset(self):
        self._next = 0
        self._works = []

    def ready(self, low_water: int):
        """All gradients at flat offsets >= low_water are final: launch complete buckets."""
        if self.world <= 1:
            return
        while self._next < len(self.buckets) and self.buckets[self._next][0] >= low_water:
            lo, hi = self.buckets[self._next]
            self._works.append(dist.all_reduce(self.grads[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))
            self._next += 1

    def finish(self) -> float:
        """Launch what is left, make the current stream wait for every bucket, return the
        grad scale (1/world) for the optimizer."""
        if self.world <= 1:
            return 1.0
        self.ready(0)
        for w in self._works:
            w.wait()
        self.reset()
        return 1.0 / self.world
