"""Rows-GEMM A/B (fp32 MFMA vs the bf16x6 split path): per-shape time AND accuracy against a
float64 product on the device, for the three rows-GEMM ops of the train step at configs[1]
(batch 16, 256x256): the pointwise forward with the BN-statistics epilogue (split path levels),
the BatchNorm-backward data gradient (the step's dominant op) and the Conv2DTranspose forward.

    UNET_HIP_LIB=tools/labbin/libunet_hip_lab.so UNET_X6=1 python tools/bench_rows.py TAG
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch  # noqa: E402
from unet_amd import ops  # noqa: E402
from unet_amd.ops import View  # noqa: E402

PEAK = 157.3
B = int(os.environ.get("B", 16))
TAG = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("UNET_X6", "0")
dev = "cuda"
DGRAD = [("enc1_block2", 256, 64, 64), ("enc2_block1", 128, 64, 128), ("enc2_block2", 128, 128, 128),
         ("enc3_block1", 64, 128, 256), ("enc3_block2", 64, 256, 256), ("enc4_block1", 32, 256, 512),
         ("enc4_block2", 32, 512, 512), ("bneck_block1", 16, 512, 1024), ("dec4_block2", 32, 512, 512),
         ("dec3_block1", 64, 512, 256), ("dec3_block2", 64, 256, 256), ("dec2_block1", 128, 256, 128),
         ("dec2_block2", 128, 128, 128), ("dec1_block1", 256, 128, 64), ("dec1_block2", 256, 64, 64)]
FWD = [("enc4_block1", 32, 256, 512), ("enc4_block2", 32, 512, 512), ("bneck_block1", 16, 512, 1024),
       ("bneck_block2", 16, 1024, 1024), ("dec4_block1", 32, 1024, 512), ("dec4_block2", 32, 512, 512)]
CONVT = [("dec4_upsample", 16, 1024, 512), ("dec3_upsample", 32, 512, 256), ("dec2_upsample", 64, 256, 128),
         ("dec1_upsample", 128, 128, 64)]


def bench(fn, iters=int(os.environ.get("ITERS", 20))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def rel(a, b):
    return float((a.double() - b).norm() / b.norm())


def emit(kind, name, m, k, n, s, fl, err):
    print(json.dumps({"tag": TAG, "op": kind, "block": name, "m": m, "k": k, "n": n, "us": round(s * 1e6, 1),
                      "tflops": round(fl / s / 1e12, 1), "frac_fp32_peak": round(fl / s / 1e12 / PEAK, 3),
                      "rel_l2_vs_f64": err}), flush=True)
    return s, fl


def main():
    g = torch.Generator(device="cpu").manual_seed(3)
    tot = {}
    for name, hw, cin, cout in DGRAD:
        m = B * hw * hw
        da = torch.randn(m, cout, generator=g).to(dev)
        z = torch.randn(m, cout, generator=g).to(dev)
        pk = (torch.randn(cin, cout, generator=g) / cin ** 0.5).to(dev)
        sc = (torch.rand(cout, generator=g) + 0.5).to(dev)
        sh = (torch.randn(cout, generator=g) * 0.1).to(dev)
        coef = (torch.randn(3 * cout, generator=g) * 0.1).to(dev)
        dy = torch.empty(m, cin, device=dev)
        dz = torch.empty(m, cout, device=dev)
        s = bench(lambda: ops.pointwise_bwd_data_bnrelu(da, z, m, cin, cout, pk, sc, sh, coef, 0.0, 7, dy, dz))
        err = rel(dy, dz.double() @ pk.double().T)
        t = emit("dgrad_bnrelu", name, m, cout, cin, s, 2.0 * m * cin * cout, err)
        tot.setdefault("dgrad_bnrelu", []).append(t)
        del da, z, dy, dz
    for name, hw, cin, cout in FWD:
        m = B * hw * hw
        y = torch.randn(m, cin, generator=g).to(dev)
        pk = (torch.randn(cin, cout, generator=g) / cin ** 0.5).to(dev)
        z = torch.empty(m, cout, device=dev)
        part = torch.zeros(ops.bn_partials_numel(m, cout), device=dev)
        s = bench(lambda: ops.pointwise_fwd(y, m, cin, cout, pk, z, part))
        err = rel(z, y.double() @ pk.double())
        tot.setdefault("pointwise_fwd", []).append(emit("pointwise_fwd", name, m, cin, cout, s, 2.0 * m * cin * cout,
                                                         err))
        del y, z, part
    for name, hw, cin, cout in CONVT:
        m = B * hw * hw
        x = torch.randn(B, hw, hw, cin, generator=g).to(dev)
        k = (torch.randn(2, 2, cout, cin, generator=g) / cin ** 0.5).to(dev)
        b = torch.randn(cout, generator=g).to(dev)
        out = torch.empty(B, 2 * hw, 2 * hw, cout, device=dev)
        v = View.plain(x)
        s = bench(lambda: ops.conv_transpose2x2_fwd(v, B, hw, hw, cout, k, b, out))
        ref = torch.einsum("nijc,abdc->niajbd", x.double(), k.double()).reshape(B, 2 * hw, 2 * hw, cout) + b.double()
        err = rel(out, ref)
        tot.setdefault("convT_fwd", []).append(emit("convT_fwd", name, m, cin, 4 * cout, s, 8.0 * m * cin * cout, err))
        del x, out
    for name, hw, cin, cout in DGRAD:  # pointwise weight gradient dW = y^T dz
        m = B * hw * hw
        y = torch.randn(m, cin, generator=g).to(dev)
        dz = torch.randn(m, cout, generator=g).to(dev)
        dpk = torch.empty(cin, cout, device=dev)
        s = bench(lambda: ops.pointwise_bwd_filter(y, dz, m, cin, cout, dpk))
        err = rel(dpk, y.double().T @ dz.double())
        tot.setdefault("pointwise_wgrad", []).append(emit("pointwise_wgrad", name, m, m, cin * cout, s,
                                                           2.0 * m * cin * cout, err))
        del y, dz
    for kind, ts in tot.items():
        us = sum(t[0] for t in ts) * 1e6
        fl = sum(t[1] for t in ts)
        print(json.dumps({"tag": TAG, "op": kind, "total_us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}))


if __name__ == "__main__":
    main()
