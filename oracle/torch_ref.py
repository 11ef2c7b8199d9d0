"""torch-CPU restatement of the reference's train step (the TF-CPU proxy of SURVEY.md §8(d)).

TEST / BASELINE INFRASTRUCTURE ONLY (see oracle/keras_ops.py header): imported by
``bench.py``'s ``cpu_baseline`` leg and by ``tests/``.  The product path never calls it.

The reference's own CPU path (TensorFlow/Keras, oneDNN) cannot run here or on the GPU box
(TensorFlow is not installed), so the CPU column of the bench is this restatement of the
identical op graph on PyTorch's CPU backend (oneDNN convolutions, channels_last, float32):
  model/u_net.py:5-26 conv_block  = depthwise 3x3 (groups=C) -> pointwise 1x1 -> BN (batch
                                    stats, eps 1e-3, momentum 0.99) -> ReLU
  model/u_net.py:63-101           = 4 x (2 blocks + MaxPool 2x2), bottleneck + Dropout, 4 x
                                    (Conv2DTranspose 2x2/2 -> concat [up, skip] -> Dropout for
                                    dec4..dec2 -> 2 blocks)
  model/u_net.py:105-112          = 1x1 head, sigmoid (1 class) / softmax
  utils/loss.py:9-29              = dice_loss (smooth 1e-7, per (b, c) over H, W, mean)
  scripts/train.py:226-231        = Keras-3 AdamW (epsilon on the un-corrected sqrt(v)) and the
                                    MeanIoU(2) confusion update on the raw probabilities.
Weights are taken in Keras layouts and permuted to torch's once.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

FILTERS = (64, 128, 256, 512)


class TorchCPUUNet:
    """The reference U-Net train step on torch-CPU (float32, channels_last)."""

    def __init__(self, weights: Dict[str, np.ndarray], num_classes: int = 1, dropout_rate: float = 0.2,
                 filters=FILTERS, lr: float = 2e-3, wd: float = 1e-4):
        self.ncls, self.rate, self.filters = num_classes, dropout_rate, tuple(filters)
        self.lr, self.wd, self.b1, self.b2, self.eps = lr, wd, 0.9, 0.999, 1e-7
        self.p: Dict[str, torch.Tensor] = {}
        self.stats: Dict[str, torch.Tensor] = {}
        for k, v in weights.items():
            t = torch.tensor(np.asarray(v, np.float32))
            if k.endswith("depthwise_kernel"):          # (3,3,C,1) -> (C,1,3,3)
                t = t.permute(2, 3, 0, 1).contiguous()
            elif k.endswith("pointwise_kernel") or k == "output_mask/kernel":  # (1,1,Ci,Co) -> (Co,Ci,1,1)
                t = t.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
            elif k.endswith("upsample/kernel"):         # (2,2,Co,Ci) -> (Ci,Co,2,2)
                t = t.permute(3, 2, 0, 1).contiguous()
            if "moving" in k:
                self.stats[k] = t
            else:
                self.p[k] = t.requires_grad_(True)
        self.m = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.iterations = 0
        self.confusion = torch.zeros(4, dtype=torch.int64)

    def _block(self, a, name):
        p = self.p
        y = F.conv2d(a, p[f"{name}_sepconv/depthwise_kernel"], padding=1, groups=a.shape[1])
        z = F.conv2d(y, p[f"{name}_sepconv/pointwise_kernel"])
        mm, mv = self.stats[f"{name}_bn/moving_mean"], self.stats[f"{name}_bn/moving_variance"]
        # training BN: batch statistics (biased variance), moving update with momentum 0.99
        z = F.batch_norm(z, mm, mv, p[f"{name}_bn/gamma"], p[f"{name}_bn/beta"], True, 0.01, 1e-3)
        return F.relu(z)

    def _drop(self, a):
        return F.dropout(a, self.rate, True) if self.rate > 0 else a

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        skips = []
        for i in range(len(self.filters)):
            h = self._block(h, f"enc{i + 1}_block1")
            h = self._block(h, f"enc{i + 1}_block2")
            skips.append(h)
            h = F.max_pool2d(h, 2)
        h = self._block(h, "bneck_block1")
        h = self._drop(self._block(h, "bneck_block2"))
        for i in range(len(self.filters)):
            st = f"dec{len(self.filters) - i}"
            u = F.conv_transpose2d(h, self.p[f"{st}_upsample/kernel"], self.p[f"{st}_upsample/bias"], stride=2)
            h = torch.cat([u, skips[len(self.filters) - 1 - i]], 1)
            if i < len(self.filters) - 1:
                h = self._drop(h)
            h = self._block(h, f"{st}_block1")
            h = self._block(h, f"{st}_block2")
        logits = F.conv2d(h, self.p["output_mask/kernel"], self.p["output_mask/bias"])
        prob = torch.sigmoid(logits) if self.ncls == 1 else torch.softmax(logits, 1)
        return prob.permute(0, 2, 3, 1)

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> float:
        for t in self.p.values():
            t.grad = None
        prob = self.forward(x)
        inter = (y * prob).sum((1, 2))
        dice = (2 * inter + 1e-7) / (y.sum((1, 2)) + prob.sum((1, 2)) + 1e-7)
        loss = 1 - dice.mean()
        loss.backward()
        with torch.no_grad():
            self.iterations += 1
            t = self.iterations
            alpha = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
            for k, w in self.p.items():
                g = w.grad
                w.sub_(w * (self.wd * self.lr))
                self.m[k].add_(g - self.m[k], alpha=1 - self.b1)
                self.v[k].add_(g * g - self.v[k], alpha=1 - self.b2)
                w.sub_(alpha * self.m[k] / (self.v[k].sqrt() + self.eps))
            # MeanIoU(2) update on raw probabilities (float -> int truncation), rows = true
            if self.ncls == 1:
                idx = y.reshape(-1).long() * 2 + prob.detach().reshape(-1).long()
                self.confusion += torch.bincount(idx, minlength=4)
        return float(loss.detach())


def cpu_info() -> Dict[str, object]:
    """Host CPU model, physical cores and the threads this process may use."""
    model, phys = "unknown", set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as f:
            for line in f:
                if ":" not in line:
                    if cur:
                        phys.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
                    continue
                k, v = (s.strip() for s in line.split(":", 1))
                cur[k] = v
                if k == "model name":
                    model = v
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = os.cpu_count() or 1
    quota = None  # cgroup v2 CPU quota of this process (cpu.max "quota period"), in CPUs
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "machine_physical_cores": len(phys) or None, "affinity_cpus": affinity,
            "machine_logical_cpus": os.cpu_count(), "cgroup_cpu_quota": quota}


def baseline_threads(info: Dict[str, object]) -> int:
    """Threads for the CPU baseline: the machine's physical cores, capped
    by what this process may actually run on (CPU affinity and the cgroup CPU quota)."""
    n = info.get("machine_physical_cores") or info.get("affinity_cpus") or 1
    n = min(int(n), int(info.get("affinity_cpus") or n))
    q = info.get("cgroup_cpu_quota")
    if q:
        n = min(n, max(1, int(q)))
    return max(1, n)


def time_train_steps(weights, size: int, batch: int, num_classes: int = 1, warmup: int = 10, steps: int = 10,
                     threads: int = 0, max_seconds: float = 300.0) -> Dict[str, object]:
    """BASELINE.md section 3 protocol: `warmup` untimed train steps, then `steps` timed steps
    of `batch` synthetic images, each timed alone; img/s from the MEDIAN step (the time budget
    max_seconds ends the timed steps early, never before 3).  Returns img/s and what was run."""
    if threads > 0:
        torch.set_num_threads(threads)
    used = torch.get_num_threads()
    torch.manual_seed(2301)
    rng = np.random.default_rng(2301)
    x = torch.from_numpy(rng.random((batch, size, size, 3), dtype=np.float32))
    if num_classes == 1:
        y = np.zeros((batch, size, size, 1), np.float32)
        for i in range(batch):
            hh, ww = int(size * rng.uniform(0.4, 0.7)), int(size * rng.uniform(0.4, 0.7))
            y0, x0 = rng.integers(0, size - hh), rng.integers(0, size - ww)
            y[i, y0:y0 + hh, x0:x0 + ww] = 1.0
    else:
        y = np.eye(num_classes, dtype=np.float32)[rng.integers(0, num_classes, (batch, size, size))]
    y = torch.from_numpy(y)
    net = TorchCPUUNet(weights, num_classes)
    t_start = time.perf_counter()
    for _ in range(max(1, warmup)):  # (the first builds the oneDNN primitives)
        net.train_step(x, y)
    t_warm = time.perf_counter() - t_start
    times = []
    t0 = time.perf_counter()
    while len(times) < steps:
        t = time.perf_counter()
        net.train_step(x, y)
        times.append(time.perf_counter() - t)
        if len(times) >= 3 and time.perf_counter() - t0 > max_seconds:
            break
    med = float(np.median(times))
    return {"value": round(batch / med, 3), "steps": len(times), "warmup": max(1, warmup),
            "median_step_s": round(med, 4), "min_step_s": round(min(times), 4), "max_step_s": round(max(times), 4),
            "warmup_seconds": round(t_warm, 2), "seconds": round(sum(times), 2), "threads": used}
