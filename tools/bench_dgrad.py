"""Per-shape timing of the BatchNorm-backward data-gradient GEMM (unet_pointwise_bwd_data_bnrelu:
dy = dz . W^T with dz formed on load from (da, z), dz stored for the weight gradient) at the 17
U-Net conv-block shapes of configs[1] (batch 16, 256x256), isolated on the device.
Reports us, TF/s, fraction of the FP32 MFMA peak and the HBM rate of the algorithmic bytes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch  # noqa: E402
from unet_amd import ops  # noqa: E402

PEAK, HBM = 157.3, 8.0
B = int(os.environ.get("B", 16))
dev = "cuda"
# (block, hw, cin, cout, dropout)
SHAPES = [("enc1_block2", 256, 64, 64, 0.0), ("enc2_block1", 128, 64, 128, 0.0), ("enc2_block2", 128, 128, 128, 0.0),
          ("enc3_block1", 64, 128, 256, 0.0), ("enc3_block2", 64, 256, 256, 0.0), ("enc4_block1", 32, 256, 512, 0.0),
          ("enc4_block2", 32, 512, 512, 0.0), ("bneck_block1", 16, 512, 1024, 0.0), ("bneck_block2", 16, 1024, 1024, 0.2),
          ("dec4_block1", 32, 1024, 512, 0.0), ("dec4_block2", 32, 512, 512, 0.0), ("dec3_block1", 64, 512, 256, 0.0),
          ("dec3_block2", 64, 256, 256, 0.0), ("dec2_block1", 128, 256, 128, 0.0), ("dec2_block2", 128, 128, 128, 0.0),
          ("dec1_block1", 256, 128, 64, 0.0), ("dec1_block2", 256, 64, 64, 0.0)]


def bench(fn, iters=20):
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


def main():
    g = torch.Generator(device="cpu").manual_seed(3)
    tot_us = tot_fl = 0.0
    for name, hw, cin, cout, drop in SHAPES:
        m = B * hw * hw
        da = torch.randn(m, cout, generator=g).to(dev)
        z = torch.randn(m, cout, generator=g).to(dev)
        pk = (torch.randn(cin, cout, generator=g) / cin ** 0.5).to(dev)
        sc = (torch.rand(cout, generator=g) + 0.5).to(dev)
        sh = (torch.randn(cout, generator=g) * 0.1).to(dev)
        coef = (torch.randn(3 * cout, generator=g) * 0.1).to(dev)
        dy = torch.empty(m, cin, device=dev)
        dz = torch.empty(m, cout, device=dev)
        s = bench(lambda: ops.pointwise_bwd_data_bnrelu(da, z, m, cin, cout, pk, sc, sh, coef, drop, 7, dy, dz))
        fl = 2.0 * m * cin * cout
        nb = 4.0 * (3 * m * cout + m * cin + cin * cout)
        t_roof = max(fl / PEAK / 1e12, nb / HBM / 1e12)
        tot_us += s * 1e6
        tot_fl += fl
        print(json.dumps({"block": name, "m": m, "cin": cin, "cout": cout, "us": round(s * 1e6, 1),
                          "tflops": round(fl / s / 1e12, 1), "frac_mfma": round(fl / s / 1e12 / PEAK, 3),
                          "tbs": round(nb / s / 1e12, 2), "frac_roof": round(t_roof / s, 3)}), flush=True)
        del da, z, dy, dz
    print(json.dumps({"total_us": round(tot_us, 1), "tflops": round(tot_fl / tot_us / 1e6, 1),
                      "frac_mfma": round(tot_fl / tot_us / 1e6 / PEAK, 3)}))


if __name__ == "__main__":
    main()
