#!/usr/bin/env python3
"""Benchmark: U-Net train step (forward + dice loss + backward + AdamW) on synthetic
256x256x3 batches, images/sec, 1..N MI355X (one process per GPU, RCCL gradient all-reduce).

BASELINE.json metric: "images/sec (train step, 256x256x3) at 1/2/4/8 MI355X"; workload =
configs[1] (batch 16 per GPU, binary, dice loss).  Weak scaling: 16 images per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

The step is the reference's `model.fit` step as scripts/train.py:227-234 compiles it: forward,
dice_loss, backward, AdamW and the MeanIoU(2) + dice_coef metric updates.

Prints ONE JSON line on rank 0.  The timed region records nothing.  `roofline` is for the
dominant kernel, timed with HIP events on its launch stream over a second pass of the same K
steps; `cpu_baseline` is the torch-CPU restatement of the same train step (oracle/torch_ref.py,
SURVEY.md 8(d)'s TF-CPU proxy) on a bounded sample, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as unet_amd/__init__.py: before HIP initialises
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

PEAK_FP32_TFLOPS = 157.3  # MI355X dense FP32 (matrix = vector rate), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# the kernel the roofline object reports (see DESIGN.md "Measurement")
ROOFLINE_OP = "unet_pointwise_fwd"


RIDGE = PEAK_FP32_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)  # flop/B


# the kernel set a PMC kernel regex (tools/pmc_traffic.py) counts, per op: the route label of
# the KernelTimer records that launch exactly those kernels
PMC_ROUTE = {"unet_pointwise_bwd_data_bnrelu": "gemm_bnbwd"}


def roofline_obj(op, s, steps):
    """Roofline object for one C-ABI op from KernelTimer totals (algorithmic flops / bytes).
    `frac` uses the op's dominant bound over all its launches; `frac_per_launch_bound` prices
    every launch against its own bound (sum of max(flops/peak, bytes/peak) over launches / time),
    so HBM-bound launches of an MFMA-labelled op are not charged at the MFMA peak."""
    sec = s["ms"] * 1e-3
    mfma = s["bytes"] == 0 or s["flops"] / s["bytes"] >= RIDGE
    if mfma:
        ach, peak, unit = s["flops"] / sec / 1e12, PEAK_FP32_TFLOPS, "TFLOP/s"
    else:
        ach, peak, unit = s["bytes"] / sec / 1e9, PEAK_HBM_GBS, "GB/s"
    traffic, tsrc = pmc_traffic(op)
    out = {"bound": "mfma" if mfma else "hbm", "kernel": op, "achieved": round(ach, 2), "peak": peak,
           "unit": unit, "frac": round(ach / peak, 4),
           "frac_per_launch_bound": round(s["t_roof_ms"] / s["ms"], 4),
           "hbm_bound_launches_per_step": s["hbm_bound_launches"] // steps,
           "traffic": traffic, "traffic_source": tsrc,
           "algorithmic_bytes_per_launch": round(s["bytes"] / s["launches"]),
           "algorithmic_flops_per_launch": round(s["flops"] / s["launches"]),
           "launches_per_step": s["launches"] // steps, "avg_launch_us": round(s["ms"] / s["launches"] * 1e3, 2)}
    r = s["routes"].get(PMC_ROUTE.get(op, "main"))
    if r:
        # the launch set the PMC regex counts: its algorithmic bytes and measured time per launch
        ab = r["bytes"] / r["launches"]
        out["pmc_launch_set"] = {"route": PMC_ROUTE.get(op, "main"), "launches_per_step": r["launches"] // steps,
                                 "algorithmic_bytes_per_launch": round(ab),
                                 "avg_launch_us": round(r["ms"] / r["launches"] * 1e3, 2),
                                 "traffic_over_algorithmic": round(traffic / ab, 3) if traffic else None,
                                 "frac_per_launch_bound": round(r["t_roof_ms"] / r["ms"], 4)}
    return out


def op_breakdown(summary):
    """Per-op time of one step, largest first, with each op's roofline fraction."""
    total = sum(d["ms"] for d in summary.values())
    rows = []
    for op, d in summary.items():
        r = roofline_obj(op, d, 1)
        rows.append({"op": op, "ms": round(d["ms"], 3), "share": round(d["ms"] / total, 4), "launches": d["launches"],
                     "bound": r["bound"], "achieved": r["achieved"], "unit": r["unit"], "frac": r["frac"]})
    rows.sort(key=lambda r: -r["ms"])
    return rows


def encoder_block_roofline(batch, size, device, reps=10, x3=True, fuse="auto"):
    """forward, training-mode conv blocks of the encoder (depthwise -> pointwise +
    BN-statistics epilogue; the BN apply + ReLU of the input is done on load, as in the train
    step) at `batch` images, each timed with HIP events around `reps` back-to-back launches (median
    of 3 groups), against
    t_roof = max(flops / peak_fp32, bytes / peak_hbm) with flops = px(18 Cin + 2 Cin Cout) and
    bytes = 4 (px (Cin + Cout) + 9 Cin + Cin Cout + 4 Cout).  Runs the train step's own kernel
    choice per block (engine.block_fwd_choice: the same launches, y stores included; block2 also
    writes the next stage's 2x2 pooling selection, which the pooled block1 reads)."""
    import torch
    from unet_amd import ops
    from unet_amd.engine import block_fwd_choice
    from unet_amd.ops import View
    g = torch.Generator(device="cpu").manual_seed(7)
    filters = (64, 128, 256, 512)
    rows, cin, h = [], 3, size
    for lvl, f in enumerate(filters):
        for blk, (ci, co) in enumerate(((cin, f), (f, f))):
            pool = lvl > 0 and blk == 0
            hh = h
            # a max-pooled input is read as the step reads it: a BN+ReLU view of the previous
            # block's 2x2 window selections (n, hh, hh, ci), written by that block (below)
            src = torch.rand((batch, hh, hh, ci), generator=g).to(device)
            sc = torch.rand(ci, generator=g).to(device) + 0.5
            sh = torch.randn(ci, generator=g).to(device) * 0.1
            ck = ci
            if lvl == 0 and blk == 0 and ci % 4:  # the engine zero-pads the image to 4 channels
                ck = (ci + 3) // 4 * 4
                src = torch.cat([src, torch.zeros(src.shape[:3] + (ck - ci,), device=device)], dim=3)
            view = View.plain(src) if (lvl == 0 and blk == 0) else View.bnrelu(src, sc, sh)
            dk = torch.randn((3, 3, ck, 1), generator=g).to(device)
            pk = (torch.randn((1, 1, ck, co), generator=g) / ci ** 0.5).to(device)
            m = batch * hh * hh
            # the train step's own kernel choice (engine.block_fwd_choice): fused launch from the
            # 64 x 64 level up, y stored unless the block's weight gradients recompute it; split
            # depthwise + pointwise launches (y always stored) below
            fused, keep_y = block_fwd_choice(view, batch, hh, hh, co, training=True, fuse=fuse)
            pkx = None  # the split-precision weight planes the engine hands the fused kernel
            if fused and x3 and ck % 16 == 0 and ck >= 64:
                pkx = torch.empty(3 * ck * co, dtype=torch.int16, device=device)
                ops.split_x3(pk, [(0, ck, co, 0)], pkx)
            ybuf = torch.empty((batch, hh, hh, ck), device=device)
            z = torch.empty((batch, hh, hh, co), device=device)
            part = torch.zeros(ops.bn_partials_numel(m, co), device=device)
            # block2 of each stage also writes the pooling selection of z for the next stage
            zsel = torch.empty((batch, hh // 2, hh // 2, co), device=device) if blk == 1 else None
            gam = (torch.rand(co, generator=g) - 0.3).to(device) if blk == 1 else None

            def run():
                if fused:
                    ops.sepconv_fwd(view, batch, hh, hh, dk, co, pk, ybuf if keep_y else None, z, part, zsel, gam,
                                    pkx)
                else:
                    ops.dwconv3x3_fwd(view, batch, hh, hh, dk, ybuf)
                    ops.pointwise_fwd(ybuf, m, ck, co, pk, z, part)
                    if zsel is not None:
                        ops.pool_select(z, batch, hh, hh, co, gam, zsel)
            for _ in range(3):
                run()
            ts = []
            for _ in range(3):  # groups of back-to-back launches: the host-side call overhead
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()     # (argument checks, ctypes) overlaps the queued kernels
                for _ in range(reps):
                    run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / reps)
            us = sorted(ts)[1]
            fl = m * (18.0 * ci + 2.0 * ci * co)
            nb = 4.0 * (m * (ci + co) + 9 * ci + ci * co + 4 * co)
            t_roof = max(fl / (PEAK_FP32_TFLOPS * 1e12), nb / (PEAK_HBM_GBS * 1e9)) * 1e6
            rows.append({"block": f"enc{lvl + 1}_block{blk + 1}", "hw": hh, "cin": ci, "cout": co,
                         "kernel": ("unet_sepconv_fwd" + (" bf16x6" if pkx is not None else "") +
                                    (" (+y store)" if keep_y else "") if fused
                                    else "dwconv3x3_fwd+pointwise_fwd") + (" +pool select" if blk == 1 else "") +
                                   (f" (input padded {ci}->{ck} ch)" if ck != ci else ""),
                         "bound": "mfma" if fl / nb >= RIDGE else "hbm", "us": round(us, 1),
                         "t_roof_us": round(t_roof, 1), "frac": round(t_roof / us, 4),
                         "tflops": round(fl / us / 1e6, 1)})
            del src, ybuf, z, part
        cin, h = f, h // 2
    mf = [r for r in rows if r["block"] >= "enc2"]
    agg = sum(r["t_roof_us"] for r in mf) / sum(r["us"] for r in mf)
    allf = sum(r["t_roof_us"] for r in rows) / sum(r["us"] for r in rows)
    torch.cuda.empty_cache()
    return {"batch": batch, "size": size, "blocks": rows, "frac_enc2_enc4": round(agg, 4),
            "frac_all": round(allf, 4), "target": 0.90}


def pmc_traffic(op):
    """HBM bytes per launch of `op` from the committed PMC summary (profiles/*traffic*.json, written
    by tools/pmc_traffic.py from FETCH_SIZE / WRITE_SIZE passes of this bench) made for THIS library
    build: the summary's lib_sha16 must equal the sha256 of the loaded libunet_hip.so.  Without
    such a summary traffic is null and the source says why."""
    import glob
    import hashlib
    from unet_amd import _lib
    try:
        with open(_lib.LIB_PATH, "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()[:16]
    except (OSError, AttributeError):
        return None, "library hash unavailable"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("op") == op and d.get("lib_sha16") == sha:
            return d["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, f"no PMC summary for this library build (lib sha256 {sha})"


def workload_config(args):
    """The BASELINE.json config whose per-GPU shape this run measures."""
    if args.size == 256 and args.num_classes == 1 and args.batch == 16:
        return "configs[1]"
    if args.size == 512 and args.num_classes == 1 and args.batch == 8:
        return "configs[3] (per-GPU shape)"
    if args.size == 256 and args.num_classes == 21 and args.batch == 8:
        return "configs[4] (per-GPU shape, batch 32 over 4 GPUs)"
    if args.size == 256 and args.num_classes == 21 and args.batch == 32:
        return "configs[4] (its whole batch of 32 on one GPU)"
    return "custom"


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


def cpu_baseline(size, ncls, batch, warmup=10, steps=10, threads=0):
    """SURVEY.md 8(d) / BASELINE.md section 3's TF-CPU proxy: the torch-CPU (oneDNN, channels_last,
    float32) restatement of the identical train step (oracle/torch_ref.py: forward, dice_loss,
    backward, Keras AdamW, MeanIoU update) on the host cores -- `warmup` untimed steps, img/s from
    the median of `steps` timed steps, threads = the machine's physical cores capped by this
    process's CPU affinity / cgroup quota (oracle/torch_ref.py baseline_threads)."""
    from oracle.torch_ref import baseline_threads, cpu_info, time_train_steps
    from unet_amd.params import init_weights, unet_variables
    info = cpu_info()
    nt = threads or baseline_threads(info)
    w = init_weights(unet_variables(3, ncls), 2301)
    r = time_train_steps(w, size, batch, ncls, warmup=warmup, steps=steps, threads=nt)
    return {"value": r["value"], "unit": "images/sec", "cores": r["threads"], "kind": "port",
            "label": "TF-CPU proxy",
            "impl": "torch-CPU restatement of the TF-CPU reference path (oneDNN, channels_last, fp32)",
            "cpu_model": info["cpu_model"], "machine_physical_cores": info["machine_physical_cores"],
            "machine_logical_cpus": info["machine_logical_cpus"], "affinity_cpus": info["affinity_cpus"],
            "cgroup_cpu_quota": info["cgroup_cpu_quota"],
            "sample": f"median of {r['steps']} timed train steps (each {batch} x {size}x{size}x3; forward + "
                      f"dice_loss + backward + AdamW + MeanIoU update) after {r['warmup']} warm-up steps; "
                      f"{r['threads']} threads; median {r['median_step_s']} s/step (min {r['min_step_s']}, "
                      f"max {r['max_step_s']})"}


def dp_info_obj(backend, exposed_ms, bucketer, steps):
    """The line's `data_parallel` object (world > 1): the backend, the all-reduce time the step
    exposes on the main stream (measured by bench.py's probe pass), the bucket layout and the ring
    volume per GPU, 2 (n - 1) / n x the gradient bytes."""
    world = bucketer.world
    grad_bytes = 4 * int(bucketer.grads.numel())
    return {"backend": backend, "collective": "all_reduce(sum) of the flat fp32 gradient buffer, "
            "bucketed, issued from the side stream as the backward completes each bucket",
            "allreduce_exposed_ms": round(float(exposed_ms), 4),
            "allreduce_exposed_definition": f"median over {steps} steps (max over ranks) of HIP-event time on "
                                            "the main stream from the end of the backward to the last bucket",
            "buckets": len(bucketer.buckets), "bucket_bytes": [4 * (hi - lo) for lo, hi in bucketer.buckets],
            "grad_bytes": grad_bytes, "world": world,
            "ring_bytes_per_gpu": round(2 * (world - 1) / world * grad_bytes)}


def result_line(args, world, dt, loss):
    """The JSON line's contract fields (rank 0): whole-job images/s over `world` ranks of
    args.batch images each (weak scaling), the time of args.steps steps (max over ranks)."""
    imgs = world * args.batch * args.steps
    return {
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
        "config": {"workload": f"{workload_config(args)}: {args.size}x{args.size}x3 "
                               f"{'binary' if args.num_classes == 1 else f'{args.num_classes}-class'} U-Net train "
                               f"step (fwd + dice_loss + bwd + AdamW + MeanIoU(2) update, dropout 0.2)",
                   "network": "U_NET separable-conv, filters 64-128-256-512, bneck 1024",
                   "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                   "seq_len": args.size * args.size, "parallelism": f"dp{world}",
                   "batchnorm": "sync" if (args.sync_bn and world > 1) else "per-replica"},
        "final_loss": round(loss, 6),
    }


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: run this same command as N torchrun ranks (one
    process per GPU) in a CHILD process and relay its exit code.  Called before anything touches
    the GPU (no torch / HIP initialisation in this parent), so no process that owns a device
    context is replaced."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--num-classes", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-warmup", type=int, default=10, help="CPU baseline warm-up steps (BASELINE.md 3)")
    ap.add_argument("--cpu-steps", type=int, default=10, help="CPU baseline timed steps (median reported)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: physical cores, capped)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-x3", action="store_true",
                    help="fp32-MFMA fused forward instead of its split-precision (bf16x6) variant (A/B)")
    ap.add_argument("--no-x6-gemm", action="store_true",
                    help="fp32-MFMA rows GEMMs (BN-backward data gradient, ConvT forward / data gradient, split-"
                         "route pointwise forward) instead of their split-precision (bf16x6) route (A/B)")
    ap.add_argument("--no-dw-fused-filter", action="store_true",
                    help="BN+ReLU-view blocks: depthwise filter gradient as its own side-stream pass instead of "
                         "inside the depthwise data-gradient pass (A/B)")
    ap.add_argument("--no-fused-bwd", action="store_true",
                    help="64-output blocks: data-gradient GEMM + side-stream weight-gradient pass instead of "
                         "the fused block backward (A/B)")
    ap.add_argument("--fuse", choices=("auto", "always"), default="auto",
                    help="fused conv forward on the levels >= 64x64 (auto) or on every level (A/B)")
    ap.add_argument("--fuse-min-pixels", type=int, default=0,
                    help="fused conv forward from levels of this many pixels per image (0: the engine's rule; A/B)")
    ap.add_argument("--fuse-min-total", type=int, default=0,
                    help="... and on smaller levels from this many pixels per launch (0: the engine's rule; A/B)")
    ap.add_argument("--recompute-y128", action="store_true",
                    help="128-output blocks too: no y store, weight gradients recompute it (A/B)")
    ap.add_argument("--recompute-y64-128", action="store_true",
                    help="the 64 -> 128 block (enc2_block1) too: no y store, recomputed (A/B)")
    ap.add_argument("--sync-bn", action="store_true",
                    help="data parallel: BatchNorm over the global batch (SyncBN) instead of per replica")
    ap.add_argument("--encoder-batch", type=int, default=32,
                    help="batch of the encoder-block roofline table (SURVEY 8(d)); 0 = skip")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    return args


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    from unet_amd import ops
    from unet_amd.dp import init_from_env
    from unet_amd.metrics import MeanIoU
    from unet_amd.model import UNetModel
    from unet_amd.optim import AdamW

    rank, world, local = init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if os.environ.get("UNET_DP_ONE_DEVICE") != "1" and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} ranks but only {torch.cuda.device_count()} visible GPU(s)")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    model = UNetModel((args.size, args.size, 3), args.num_classes, dropout_rate=0.2, device=device)
    # as scripts/train.py:227-234 compiles it: dice_loss, metrics MeanIoU(2) + dice_coef, so the
    # MeanIoU confusion update runs inside every timed step
    model.compile(AdamW(learning_rate=2e-3, weight_decay=1e-4), "dice_loss",
                  metrics=[MeanIoU(num_classes=2, name="mean_io_u", device=device), "dice_coef"])
    if world > 1:
        model.enable_data_parallel(sync_bn=args.sync_bn)
    model.engine.use_x3 = not args.no_x3
    model.engine.x6_gemm = not args.no_x6_gemm
    model.engine.dw_fused_filter = not args.no_dw_fused_filter
    model.engine.fuse_block_bwd = not args.no_fused_bwd
    model.engine.fuse_sepconv = args.fuse
    if args.fuse_min_pixels:
        model.engine.fuse_min_pixels = args.fuse_min_pixels
    if args.fuse_min_total:
        model.engine.fuse_min_total = args.fuse_min_total
    if args.recompute_y128:
        model.engine.recompute_y_couts = (64, 128)
    elif args.recompute_y64_128:
        model.engine.recompute_y_couts = (64, (64, 128))
    x, y = synthetic_batch(args.batch, args.size, args.size, args.num_classes, 2301 + rank, device)

    for _ in range(args.warmup):
        model.train_step(x, y)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    # per-op breakdown: one untimed single-stream step with every C-ABI op bracketed by HIP
    # events on its launch stream; its largest op is the one the roofline object reports
    breakdown, dominant = None, ROOFLINE_OP
    if not args.no_roofline:
        bt = ops.KernelTimer(None)
        ops.TIMER = bt
        overlap = model.engine.overlap
        model.engine.overlap = False  # single stream: per-op times not inflated by the side stream
        model.train_step(x, y)
        model.engine.overlap = overlap
        ops.TIMER = None
        breakdown = op_breakdown(bt.summary())
        dominant = breakdown[0]["op"]

    # the timed region: K steps, nothing recorded inside it
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = model.train_step(x, y)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    loss = float(res[0].item())
    # the MeanIoU of the timed steps (warm-up + K), read before the roofline / all-reduce probe
    # passes below train further, so 1-GPU and N-GPU lines report the same quantity
    miou = model.mean_iou.result()

    # roofline pass: the same K steps again (same streams, same overlap) with the dominant
    # kernel's launches bracketed by HIP events on the stream each is issued on
    timer, dt_roof = None, None
    if not args.no_roofline:
        timer = ops.KernelTimer([dominant])
        ops.TIMER = timer
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            model.train_step(x, y)
        torch.cuda.synchronize()
        dt_roof = time.perf_counter() - t1
        ops.TIMER = None

    # data parallel: a separate pass of K steps measuring the all-reduce time the step exposes on
    # the main stream (from the end of the backward's launches to the last bucket's completion)
    dp_info = None
    if world > 1:
        probe = []
        model.dp_probe = probe
        for _ in range(args.steps):
            model.train_step(x, y)
        torch.cuda.synchronize()
        model.dp_probe = None
        ex = sorted(a.elapsed_time(b) for a, b in probe)
        t = torch.tensor([ex[len(ex) // 2]], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dp_info = dp_info_obj(dist.get_backend(), float(t.item()), model.bucketer, args.steps)

    out = None
    if rank == 0:
        out = result_line(args, world, dt, loss)
        if timer is not None:
            s = timer.summary().get(dominant)
            if s:
                out["roofline"] = roofline_obj(dominant, s, args.steps)
                out["roofline"]["timing"] = (f"separate pass of {args.steps} steps after the timed region "
                                             f"({dt_roof / args.steps * 1e3:.3f} ms/step with events)")
                out["op_breakdown"] = breakdown[:8]
        if dp_info is not None:
            out["data_parallel"] = dp_info
        if model.mean_iou is not None:
            out["mean_io_u"] = round(miou, 6)
        if not args.no_roofline and world == 1 and args.encoder_batch > 0:
            del model
            torch.cuda.empty_cache()
            out["encoder_blocks"] = encoder_block_roofline(args.encoder_batch, args.size, device, x3=not args.no_x3,
                                                           fuse=args.fuse)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.size, args.num_classes, args.batch, args.cpu_warmup,
                                               args.cpu_steps, args.cpu_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
