"""Per-shape timing of the pointwise / transposed-conv GEMM entry points at the U-Net's
configs[1] shapes (batch 16, 256x256), reporting TFLOP/s and fraction of the FP32 MFMA peak."""
import os, sys, json, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from unet_amd import ops
from unet_amd.ops import View

PEAK = 157.3
B = int(os.environ.get("B", 16))
dev = "cuda"
def t(*shape): return torch.randn(*shape, device=dev)

def bench(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3

blocks = [(256, 3, 64), (256, 64, 64), (128, 64, 128), (128, 128, 128), (64, 128, 256), (64, 256, 256),
          (32, 256, 512), (32, 512, 512), (16, 512, 1024), (16, 1024, 1024), (32, 1024, 512), (64, 512, 256),
          (128, 256, 128), (256, 128, 64)]
res = []
for hw, cin, cout in blocks:
    m = B * hw * hw
    y, pk, z = t(m, cin), t(cin, cout) * 0.1, t(m, cout)
    part = torch.zeros(ops.bn_partials_numel(m, cout), device=dev)
    dz, dy, dpk = t(m, cout), t(m, cin), t(cin, cout)
    fl = 2.0 * m * cin * cout
    r = {"hw": hw, "cin": cin, "cout": cout}
    for name, fn in [("fwd", lambda: ops.pointwise_fwd(y, m, cin, cout, pk, z, part)),
                     ("dgrad", lambda: ops.pointwise_bwd_data(dz, m, cin, cout, pk, dy)),
                     ("wgrad", lambda: ops.pointwise_bwd_filter(y, dz, m, cin, cout, dpk))]:
        s = bench(fn)
        r[name] = (round(s * 1e6, 1), round(fl / s / 1e12, 1))
    res.append(r)
    print(json.dumps(r), flush=True)
for hw, cin, cout in [(16, 1024, 512), (32, 512, 256), (64, 256, 128), (128, 128, 64)]:
    m = B * hw * hw
    z, sc, sh = t(m, cin), torch.rand(cin, device=dev), t(cin) * 0.1
    v = View.bnrelu(z, sc, sh)
    k, b = t(2, 2, cout, cin) * 0.05, t(cout)
    out, dout, dx, dk, db = t(B, 2 * hw, 2 * hw, cout), t(B, 2 * hw, 2 * hw, cout), t(B, hw, hw, cin), t(2, 2, cout, cin), t(cout)
    fl = 8.0 * m * cin * cout
    s1 = bench(lambda: ops.conv_transpose2x2_fwd(v, B, hw, hw, cout, k, b, out))
    s2 = bench(lambda: ops.conv_transpose2x2_bwd(v, B, hw, hw, cout, k, dout, dx, dk, db))
    print(json.dumps({"convT": (hw, cin, cout), "fwd": (round(s1 * 1e6, 1), round(fl / s1 / 1e12, 1)),
                      "bwd(data+filter+bias)": (round(s2 * 1e6, 1), round(2 * fl / s2 / 1e12, 1))}), flush=True)
