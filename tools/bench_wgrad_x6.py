"""Weight-gradient GEMMs, fp32-MFMA vs split-precision (bf16x6, both operands split as staged) on the
128 x 128-tile shapes of the train step at configs[1] (batch 16): the pointwise weight gradient
dW = y^T dz and the Conv2DTranspose kernel gradient (+ bias).  Needs the LAB library (the switch is
the lab knob UNET_WGRAD_X6, read per launch):

    UNET_HIP_LIB=tools/labbin/libunet_hip_lab.so python tools/bench_wgrad_x6.py [TAG]
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
TAG = sys.argv[1] if len(sys.argv) > 1 else "wx6"
PW = [("enc2_block2", 128, 128, 128), ("enc3_block1", 64, 128, 256), ("enc3_block2", 64, 256, 256),
      ("enc4_block1", 32, 256, 512), ("enc4_block2", 32, 512, 512), ("bneck_block1", 16, 512, 1024),
      ("bneck_block2", 16, 1024, 1024), ("dec4_block1", 32, 1024, 512), ("dec3_block1", 64, 512, 256),
      ("dec2_block1", 128, 256, 128), ("dec2_block2", 128, 128, 128)]
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


def both(fn):
    res = {}
    for key, knob in (("f32", "0"), ("x6", "1")):
        os.environ["UNET_WGRAD_X6"] = knob
        res[key] = (bench(fn), None)
        res[key] = (res[key][0], fn())
    return res


def main():
    g = torch.Generator(device="cpu").manual_seed(5)
    tot = {"f32": 0.0, "x6": 0.0}
    for name, hw, cin, cout in PW:
        m = B * hw * hw
        y = torch.randn(m, cin, generator=g).to("cuda")
        dz = torch.randn(m, cout, generator=g).to("cuda")

        def run():
            out = torch.empty(cin, cout, device="cuda")
            ops.pointwise_bwd_filter(y, dz, m, cin, cout, out)
            return out
        res = both(run)
        ref = y.double().T @ dz.double()
        fl = 2.0 * m * cin * cout
        for k in tot:
            tot[k] += res[k][0]
        print(json.dumps({"tag": TAG, "op": "pointwise_wgrad", "block": name, "m": m, "p": cin, "q": cout,
                          "us_f32": round(res["f32"][0] * 1e6, 1), "us_x6": round(res["x6"][0] * 1e6, 1),
                          "frac_f32": round(fl / res["f32"][0] / 1e12 / PEAK, 3),
                          "frac_x6": round(fl / res["x6"][0] / 1e12 / PEAK, 3),
                          "rel_f32": rel(res["f32"][1], ref), "rel_x6": rel(res["x6"][1], ref)}), flush=True)
        del y, dz
    for name, hw, cin, cout in CONVT:
        m = B * hw * hw
        z = torch.randn(B, hw, hw, cin, generator=g).to("cuda")
        sc = (torch.rand(cin, generator=g) + 0.5).to("cuda")
        sh = (torch.randn(cin, generator=g) * 0.1).to("cuda")
        v = View.bnrelu(z, sc, sh)
        k = (torch.randn(2, 2, cout, cin, generator=g) * 0.1).to("cuda")
        dout = torch.randn(B, 2 * hw, 2 * hw, cout, generator=g).to("cuda")

        def run():
            dk = torch.empty(2, 2, cout, cin, device="cuda")
            db = torch.empty(cout, device="cuda")
            ops.conv_transpose2x2_bwd(v, B, hw, hw, cout, k, dout, None, dk, db)
            return dk
        res = both(run)
        x = torch.relu(z.double() * sc.double() + sh.double())
        ref = torch.einsum("niajbd,nijc->abdc", dout.double().reshape(B, hw, 2, hw, 2, cout), x)
        fl = 8.0 * m * cin * cout
        for kk in tot:
            tot[kk] += res[kk][0]
        print(json.dumps({"tag": TAG, "op": "convT_wgrad", "block": name, "m": m, "p": 4 * cout, "q": cin,
                          "us_f32": round(res["f32"][0] * 1e6, 1), "us_x6": round(res["x6"][0] * 1e6, 1),
                          "frac_f32": round(fl / res["f32"][0] / 1e12 / PEAK, 3),
                          "frac_x6": round(fl / res["x6"][0] / 1e12 / PEAK, 3),
                          "rel_f32": rel(res["f32"][1], ref), "rel_x6": rel(res["x6"][1], ref)}), flush=True)
        del z, dout
    print(json.dumps({"tag": TAG, "total_us_f32": round(tot["f32"] * 1e6, 1), "total_us_x6": round(tot["x6"] * 1e6, 1)}))


if __name__ == "__main__":
    main()
