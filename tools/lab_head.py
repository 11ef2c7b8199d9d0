"""Lab: the multi-class head kernels alone at configs[4]'s per-GPU shape (batch 8, 256x256, 64 ->
21 classes): forward, dice sums, fused backward, and the backward under knock-outs
(UNET_HEAD_KO bits, lab library: 1 no loss_grad, 2 no input loads, 4 no dx stores, 8 no staging
loads, 16 no db sums, 32 no phase-2 products, 64 no phase 1).
usage: UNET_HIP_LIB=tools/labbin/libunet_hip_lab.so python tools/lab_head.py KO [KO ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]


def child(ko):
    import torch
    from unet_amd import ops
    from unet_amd.ops import View
    n, h, w, c, k = 8, 256, 256, 64, 21
    g = torch.Generator(device="cpu").manual_seed(3)
    z = torch.randn(n, h, w, c, generator=g).cuda()
    sc, sh = (torch.rand(c, generator=g) + 0.5).cuda(), (torch.randn(c, generator=g) * 0.1).cuda()
    v = View.bnrelu(z, sc, sh)
    W, b = (torch.randn(c * k, generator=g) * 0.1).cuda(), torch.zeros(k).cuda()
    prob = torch.empty(n, h, w, k, device="cuda")
    yt = torch.nn.functional.one_hot(torch.randint(0, k, (n, h, w), generator=g), k).float().cuda()
    sums, res = torch.empty(n * k * 3, device="cuda"), torch.empty(3, device="cuda")
    dx, dk, db = torch.empty_like(z), torch.empty(c * k, device="cuda"), torch.empty(k, device="cuda")

    def t(fn, reps=20):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / reps)
        return round(sorted(ts)[2], 1)
    r = {"ko": ko}
    if ko == 0:
        r["fwd_us"] = t(lambda: ops.head_fwd(v, n, h, w, k, W, b, prob))
        r["dice_us"] = t(lambda: ops.dice_fwd(yt, prob, n, h * w, k, 1e-7, sums, res))
    ops.head_fwd(v, n, h, w, k, W, b, prob)
    ops.dice_fwd(yt, prob, n, h * w, k, 1e-7, sums, res)
    r["bwd_us"] = t(lambda: ops.head_bwd(v, n, h, w, k, W, prob, yt, sums, 1e-7, 0, dx, dk, db))
    mb = (z.numel() * 8 + prob.numel() * 8) / 1e6
    r["bwd_MB"] = round(mb, 1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(int(sys.argv[2]))
    else:
        for ko in sys.argv[1:] or ["0"]:  # the knob is read once per process: one child per value
            env = dict(os.environ, UNET_HEAD_KO=ko)
            subprocess.run([sys.executable, __file__, "--child", ko], env=env, check=True)
