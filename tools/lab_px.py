"""Lab: the persistent split-precision sepconv forward (sepconv_px.hip, schedule AUTO) against the
one-tile-per-block register-A kernel (schedule RK1) on the short-K shapes (schedule RK: every supported shape): z / y / pooling
selection compared (bitwise expected: same products, same order) and the BN statistics partials
(per tile, combined in a different order: ~1e-6 relative), and both timed with HIP events around
back-to-back launches (median of 3 groups of 10).  With the lab library (UNET_HIP_LIB=
tools/labbin/libunet_hip_lab.so) UNET_PX_PD / UNET_PX_BPC select the prefetch depth / blocks per CU.
usage: python tools/lab_px.py [N] [check|time|both]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch

from unet_amd import ops
from unet_amd.ops import View

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
WHAT = sys.argv[2] if len(sys.argv) > 2 else "both"
g = torch.Generator(device="cpu").manual_seed(3)
dev = "cuda"


def rnd(*s, scale=1.0):
    return (torch.rand(s, generator=g) * 2 - 1).mul_(scale).to(dev)


SHAPES = [  # name, mode, n, hw, cin(c0, c1), cout, y, zsel, drop, stats
    ("enc1_block2", "bnrelu", N, 256, (64, 0), 64, False, True, 0.0, True),
    ("enc2_block1", "bnrelu", N, 128, (64, 0), 128, True, False, 0.0, True),
    ("enc2_block2", "bnrelu", N, 128, (128, 0), 128, True, True, 0.0, True),
    ("dec1_block1", "concat", N // 2, 256, (64, 64), 64, False, False, 0.0, True),
    ("dec1_block2", "bnrelu", N // 2, 256, (64, 0), 64, False, False, 0.0, True),
    ("dec2_block2", "bnrelu", N // 2, 128, (128, 0), 128, True, False, 0.0, True),
    ("dec2_b1_drop", "concat", 2, 128, (64, 64), 128, True, False, 0.2, True),
    ("plain_infer", "plain", 2, 64, (64, 0), 64, False, True, 0.0, False),
]


def run_shape(name, mode, n, hw, cc, cout, wy, sel, drop, stats):
    c0, c1 = cc
    cin = c0 + c1
    src0 = rnd(n, hw, hw, c0)
    sc0, sh0 = rnd(c0, scale=0.5) + 1.0, rnd(c0, scale=0.2)
    if mode == "bnrelu":
        v = View.bnrelu(src0, sc0, sh0)
    elif mode == "plain":
        v = View.plain(src0)
    else:
        src1 = rnd(n, hw, hw, c1)
        v = View.concat(src0, src1, rnd(c1, scale=0.5) + 1.0, rnd(c1, scale=0.2))
    if drop:
        v = v.dropout(drop, 12345)
    dk = rnd(3, 3, cin, 1, scale=0.5)
    pk = rnd(1, 1, cin, cout, scale=1.0 / cin ** 0.5)
    pkx = torch.empty(3 * cin * cout, dtype=torch.int16, device=dev)
    ops.split_x3(pk, [(0, cin, cout, 0)], pkx)
    m = n * hw * hw
    gam = rnd(cout) if sel else None
    outs = {}
    for sch in (ops.SEPCONV_RK1, ops.SEPCONV_RK):
        y = torch.full((n, hw, hw, cin), float("nan"), device=dev) if wy else None
        z = torch.full((n, hw, hw, cout), float("nan"), device=dev)
        part = torch.zeros(ops.bn_partials_numel(m, cout), device=dev) if stats else None
        zs = torch.full((n, hw // 2, hw // 2, cout), float("nan"), device=dev) if sel else None
        old = ops.sepconv_set_schedule(sch)

        def f():
            ops.sepconv_fwd(v, n, hw, hw, dk, cout, pk, y, z, part, zs, gam, pkx)
        f()
        torch.cuda.synchronize()
        rec = {"z": z.clone(), "y": None if y is None else y.clone(), "part": None if part is None else part.clone(),
               "zs": None if zs is None else zs.clone()}
        if WHAT in ("time", "both"):
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 100.0)
            rec["us"] = sorted(ts)[1]
        ops.sepconv_set_schedule(old)
        outs[sch] = rec
    a, b = outs[ops.SEPCONV_RK1], outs[ops.SEPCONV_RK]
    res = {"shape": name, "n": n, "hw": hw, "cin": cin, "cout": cout}
    res["z_bitwise"] = bool(torch.equal(a["z"], b["z"]))
    res["z_maxrel"] = float(((a["z"] - b["z"]).abs().max() / a["z"].abs().max()).item())
    if wy:
        res["y_bitwise"] = bool(torch.equal(a["y"], b["y"]))
    if sel:
        res["zsel_bitwise"] = bool(torch.equal(a["zs"], b["zs"]))
    if stats:
        nb = m // 128 * cout * 2
        pa, pb = a["part"][:nb].view(-1, cout, 2), b["part"][:nb].view(-1, cout, 2)
        res["stats_mean_maxabs"] = float((pa[..., 0] - pb[..., 0]).abs().max().item())
        res["stats_m2_maxrel"] = float(((pa[..., 1] - pb[..., 1]).abs() / pa[..., 1].abs().clamp_min(1e-20)).max().item())
    if "us" in a:
        rd = 4.0 * m * cin
        wr = 4.0 * (m * cout + (m * cin if wy else 0) + (m // 4 * cout if sel else 0))
        res.update({"us_rk1": round(a["us"], 1), "us_px": round(b["us"], 1), "speedup": round(a["us"] / b["us"], 3),
                    "tbps_px": round((rd + wr) / b["us"] / 1e6, 2)})
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    env = {k: os.environ.get(k) for k in ("UNET_HIP_LIB", "UNET_PX_PD", "UNET_PX_BPC")}
    print(json.dumps({"env": env, "N": N}), flush=True)
    for s in SHAPES:
        run_shape(*s)
