"""Read-bandwidth probe for the binary head forward (head_fwd_bin_kernel) against a plain read
(torch sum) of the same 16x256x256x64 fp32 tensor: HIP-event timing, median of 20."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from unet_amd import ops
from unet_amd.ops import View

n, h, w, c = 16, 256, 256, 64
z = torch.randn((n, h, w, c), device="cuda")
sc, sh = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.1
k, b = torch.randn((1, 1, c, 1), device="cuda") * 0.1, torch.zeros(1, device="cuda")
prob = torch.empty((n, h, w, 1), device="cuda")


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


nb = z.numel() * 4
for name, fn in [("head_fwd bnrelu", lambda: ops.head_fwd(View.bnrelu(z, sc, sh), n, h, w, 1, k, b, prob)),
                 ("head_fwd plain", lambda: ops.head_fwd(View.plain(z), n, h, w, 1, k, b, prob)),
                 ("torch sum", lambda: z.sum()),
                 ("torch copy", lambda: prob.copy_(z[..., :1]))]:
    us = timed(fn)
    print(f"{name:18s} {us:8.1f} us  {nb / us / 1e3:7.1f} GB/s (of the 268 MB input)")
