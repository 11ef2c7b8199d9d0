#!/usr/bin/env python3
"""Benchmark: U-Net train step (forward + dice loss + backward + AdamW) on synthetic
256x256x3 batches, images/sec, 1..N MI355X (one process per GPU, RCCL gradient all-reduce).

BASELINE.json metric: "images/sec (train step, 256x256x3) at 1/2/4/8 MI355X"; workload =
configs[1] (batch 16 per GPU, binary, dice loss).  Weak scaling: 16 images per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel, timed with HIP events
on its launch stream over the timed region; `cpu_baseline` is the NumPy oracle train step
(oracle/unet_ref.py) on a bounded sample, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

PEAK_FP32_TFLOPS = 157.3  # MI355X dense FP32 (matrix = vector rate), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# the kernel the roofline object reports (see DESIGN.md "Measurement")
ROOFLINE_OP = "unet_pointwise_fwd"


def pmc_traffic(op):
    """HBM bytes per launch of `op` from the newest committed PMC summary (profiles/*_traffic.json,
    written by tools/pmc_traffic.py from FETCH_SIZE / WRITE_SIZE passes of this bench)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("op") == op:
            return d["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def synthetic_batch(n, h, w, ncls, seed, device):
    import numpy as np
    import torch
    rng = np.random.default_rng(seed)
    x = rng.random((n, h, w, 3), dtype=np.float32)  # U[0,1): images after rescale=1/255
    if ncls == 1:  # ID-card-like quads, ~30 % foreground
        y = np.zeros((n, h, w, 1), np.float32)
        for i in range(n):
            hh, ww = int(h * rng.uniform(0.4, 0.7)), int(w * rng.uniform(0.4, 0.7))
            y0, x0 = rng.integers(0, h - hh), rng.integers(0, w - ww)
            y[i, y0:y0 + hh, x0:x0 + ww] = 1.0
    else:
        y = np.eye(ncls, dtype=np.float32)[rng.integers(0, ncls, (n, h, w))]
    return torch.from_numpy(x).to(device), torch.from_numpy(y).to(device)


def cpu_baseline(size, ncls, n_img=2):
    """NumPy oracle train step (float32), batch 1, n_img steps; img/s."""
    import numpy as np
    from oracle.unet_ref import UNetOracle
    from unet_amd.params import init_weights, unet_variables
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        threads = 1
    specs = unet_variables(3, ncls)
    p = init_weights(specs, 1)
    opt = {s.name: (np.zeros(s.shape, np.float32), np.zeros(s.shape, np.float32)) for s in specs if s.trainable}
    o = UNetOracle(ncls, 0.2)
    seeds = {s: i for i, s in enumerate(("bneck_dropout", "dec4_dropout", "dec3_dropout", "dec2_dropout"))}
    rng = np.random.default_rng(0)
    t0 = time.perf_counter()
    for i in range(n_img):
        x = rng.random((1, size, size, 3), dtype=np.float32)
        y = (rng.random((1, size, size, ncls)) > 0.5).astype(np.float32)
        _, _, _, p, opt, _ = o.train_step(p, opt, x, y, i + 1, 2e-3, 1e-4, drop_seeds=seeds)
    dt = time.perf_counter() - t0
    return {"value": round(n_img / dt, 4), "unit": "images/sec", "cores": int(threads), "kind": "port",
            "sample": f"{n_img} train steps of batch 1 at {size}x{size}x3 (NumPy oracle, float32, "
                      f"forward+dice+backward+AdamW) on the host CPU"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--num-classes", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from unet_amd import ops
    from unet_amd.dp import init_from_env
    from unet_amd.model import UNetModel
    from unet_amd.optim import AdamW

    rank, world, local = init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    model = UNetModel((args.size, args.size, 3), args.num_classes, dropout_rate=0.2, device=device)
    model.compile(AdamW(learning_rate=2e-3, weight_decay=1e-4), "dice_loss")
    if world > 1:
        model.enable_data_parallel()
    x, y = synthetic_batch(args.batch, args.size, args.size, args.num_classes, 2301 + rank, device)

    for _ in range(args.warmup):
        model.train_step(x, y)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    timer = None
    if not args.no_roofline:
        timer = ops.KernelTimer([ROOFLINE_OP])
        ops.TIMER = timer
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = model.train_step(x, y)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    ops.TIMER = None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    loss = float(res[0].item())

    out = None
    if rank == 0:
        imgs = world * args.batch * args.steps
        out = {
            "metric": "images/sec (train step, 256x256x3)",
            "value": round(imgs / dt, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (x~U[0,1) NHWC, quad masks ~30% fg), random-init Keras-glorot weights",
            "config": {"workload": f"configs[1]: {args.size}x{args.size}x3 binary U-Net train step "
                                   f"(fwd + dice_loss + bwd + AdamW, dropout 0.2)",
                       "model": "U_NET separable-conv, filters 64-128-256-512, bneck 1024",
                       "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                       "seq_len": args.size * args.size, "parallelism": f"dp{world}"},
            "final_loss": round(loss, 6),
        }
        if timer is not None:
            s = timer.summary().get(ROOFLINE_OP)
            if s:
                avg_ms = s["ms"] / s["launches"]
                ach = s["flops"] / (s["ms"] * 1e-3) / 1e12
                traffic, tsrc = pmc_traffic(ROOFLINE_OP)
                out["roofline"] = {"bound": "mfma", "kernel": ROOFLINE_OP, "achieved": round(ach, 2),
                                   "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                                   "frac": round(ach / PEAK_FP32_TFLOPS, 4), "traffic": traffic,
                                   "traffic_source": tsrc,
                                   "algorithmic_bytes_per_launch": round(s["bytes"] / s["launches"]),
                                   "launches_per_step": s["launches"] // args.steps,
                                   "avg_launch_us": round(avg_ms * 1e3, 2),
                                   "algorithmic_gflop_per_step": round(s["flops"] / args.steps / 1e9, 3)}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.size, args.num_classes)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
