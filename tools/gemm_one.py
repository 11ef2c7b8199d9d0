"""Run one GEMM entry point repeatedly (for rocprofv3 --pmc passes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from unet_amd import ops
kind = sys.argv[1]; m, cin, cout = (int(v) for v in sys.argv[2:5]); iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
y, pk, z = torch.randn(m, cin, device="cuda"), torch.randn(cin, cout, device="cuda") * 0.1, torch.empty(m, cout, device="cuda")
part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
dz, dy, dpk = torch.randn(m, cout, device="cuda"), torch.empty(m, cin, device="cuda"), torch.empty(cin, cout, device="cuda")
for _ in range(iters):
    if kind == "fwd": ops.pointwise_fwd(y, m, cin, cout, pk, z, part)
    elif kind == "dgrad": ops.pointwise_bwd_data(dz, m, cin, cout, pk, dy)
    else: ops.pointwise_bwd_filter(y, dz, m, cin, cout, dpk)
torch.cuda.synchronize()
