"""Conv2DTranspose forward / data-gradient timing at the U-Net's decoder shapes (configs[1]:
batch 16), for tile sweeps: run once per UNET_ROWS_CFG value (read once per process).
usage: UNET_ROWS_CFG=BN,BK python tools/bench_convt.py"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from unet_amd import ops
from unet_amd.ops import View

PEAK = 157.3
B = int(os.environ.get("B", 16))
dev = "cuda"


def t(*shape):
    return torch.randn(*shape, device=dev)


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


tot_f = tot_b = 0.0
for hw, cin, cout in [(16, 1024, 512), (32, 512, 256), (64, 256, 128), (128, 128, 64)]:
    m = B * hw * hw
    z, sc, sh = t(m, cin), torch.rand(cin, device=dev), t(cin) * 0.1
    v = View.bnrelu(z, sc, sh)
    k, b = t(2, 2, cout, cin) * 0.05, t(cout)
    out, dout, dx = t(B, 2 * hw, 2 * hw, cout), t(B, 2 * hw, 2 * hw, cout), t(B, hw, hw, cin)
    fl = 8.0 * m * cin * cout
    s1 = bench(lambda: ops.conv_transpose2x2_fwd(v, B, hw, hw, cout, k, b, out))
    s2 = bench(lambda: ops.conv_transpose2x2_bwd(v, B, hw, hw, cout, k, dout, dx, None, None))
    tot_f += s1
    tot_b += s2
    print(json.dumps({"cfg": os.environ.get("UNET_ROWS_CFG", "default"), "convT": (hw, cin, cout),
                      "fwd_us": round(s1 * 1e6, 1), "fwd_tf": round(fl / s1 / 1e12, 1),
                      "dgrad_us": round(s2 * 1e6, 1), "dgrad_tf": round(fl / s2 / 1e12, 1)}), flush=True)
print(json.dumps({"cfg": os.environ.get("UNET_ROWS_CFG", "default"), "fwd_total_us": round(tot_f * 1e6, 1),
                  "dgrad_total_us": round(tot_b * 1e6, 1)}), flush=True)
