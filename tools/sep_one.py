"""Run the fused sepconv forward (or the split dw + pw pair) on one shape repeatedly, for
rocprofv3 --pmc passes.  usage: sep_one.py MODE H W CIN COUT [iters] [split|x3]   (N images: env N,
default 16; x3 = the split-precision variant with pre-split weight planes, as the train step runs
it at channels % 16 == 0)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from unet_amd import ops
mode, h, w, C, cout = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
opt = sys.argv[7] if len(sys.argv) > 7 else ""
N = int(os.environ.get("N", 16))
if os.environ.get("SCHED"):  # 3 = RK1 (one tile per block), 0 = AUTO (persistent where it applies)
    ops.sepconv_set_schedule(int(os.environ["SCHED"]))
big = 2 if mode == 2 else 1
src = torch.randn(N, big * h, big * w, C, device="cuda")
sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
v = ops.View.plain(src) if mode == 0 else (ops.View.pool_bnrelu(src, sc, sh) if mode == 2 else ops.View.bnrelu(src, sc, sh))
m = N * h * w
dk = torch.randn(3, 3, C, 1, device="cuda")
pk = torch.randn(1, 1, C, cout, device="cuda") * 0.05
pkx = None
if opt == "x3":
    pkx = torch.empty(3 * C * cout, dtype=torch.int16, device="cuda")
    ops.split_x3(pk, [(0, C, cout, 0)], pkx)
y = torch.empty(N, h, w, C, device="cuda")
z = torch.empty(N, h, w, cout, device="cuda")
part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
# POOL=1: also the 2x2 max-pool selection epilogue (an encoder stage's block2, as the step runs it)
zsel = torch.empty(N, h // 2, w // 2, cout, device="cuda") if os.environ.get("POOL") == "1" else None
gam = torch.rand(cout, device="cuda") - 0.3 if zsel is not None else None
for _ in range(iters):
    if opt == "split":
        ops.dwconv3x3_fwd(v, N, h, w, dk, y)
        ops.pointwise_fwd(y, m, C, cout, pk, z, part)
    else:
        ops.sepconv_fwd(v, N, h, w, dk, cout, pk, y, z, part, zsel, gam, pkx=pkx)
torch.cuda.synchronize()
