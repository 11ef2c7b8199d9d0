"""Weight gradients of the conv blocks the fused pass covers, at configs[1] shapes (batch 16,
256x256), isolated on the device: the separate route (pointwise_bwd_filter over a stored y +
dwconv3x3_bwd_filter over the view) against unet_sepconv_bwd_filter (one pass, y recomputed)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch  # noqa: E402
from unet_amd import ops  # noqa: E402
from unet_amd.ops import View  # noqa: E402

B = int(os.environ.get("B", 16))
dev = "cuda"
# (block, hw, (c0, c1) of the view, cout)
SHAPES = [("enc1_block2", 256, (64, 0), 64), ("dec1_block1", 256, (64, 64), 64), ("dec1_block2", 256, (64, 0), 64)]


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    g = torch.Generator(device="cpu").manual_seed(5)
    tot = [0.0, 0.0]
    for name, hw, (c0, c1), cout in SHAPES:
        n, C = B, c0 + c1
        m = n * hw * hw
        aff = lambda c: ((torch.rand(c, generator=g) + 0.5).to(dev), (torch.randn(c, generator=g) * 0.1).to(dev))
        src0 = torch.randn(n, hw, hw, c0, generator=g).to(dev)
        if c1:
            v = View.concat(src0, torch.randn(n, hw, hw, c1, generator=g).to(dev), *aff(c1))
        else:
            v = View.bnrelu(src0, *aff(c0))
        dk = torch.randn(3, 3, C, 1, generator=g).to(dev)
        y, dy = torch.randn(m, C, generator=g).to(dev), torch.randn(m, C, generator=g).to(dev)
        dz = torch.randn(m, cout, generator=g).to(dev)
        ddk, dpk = torch.empty(3, 3, C, 1, device=dev), torch.empty(1, 1, C, cout, device=dev)

        def old():
            ops.pointwise_bwd_filter(y, dz, m, C, cout, dpk)
            ops.dwconv3x3_bwd_filter(v, n, hw, hw, dy, ddk)

        def new():
            ops.sepconv_bwd_filter(v, n, hw, hw, dk, dy, dz, cout, ddk, dpk)
        t0, t1 = bench(old), bench(new)
        tot[0] += t0
        tot[1] += t1
        print(json.dumps({"block": name, "m": m, "cin": C, "cout": cout, "separate_us": round(t0, 1),
                          "fused_us": round(t1, 1), "fused_tbs": round(4.0 * m * (2 * C + cout) / t1 / 1e6, 2)}),
              flush=True)
        del src0, y, dy, dz
    print(json.dumps({"separate_total_us": round(tot[0], 1), "fused_total_us": round(tot[1], 1)}))


if __name__ == "__main__":
    main()
