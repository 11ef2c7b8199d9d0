"""Per-op timing on the U-Net's layer shapes (batch 16, 256x256 input) with achieved algorithmic
GB/s (and TF/s for GEMMs): the table that says which kernel is furthest from its roofline."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from unet_amd import ops

N = 16
SHAPES = [  # mode, h, w, c0, c1, cout
    (1, 256, 256, 64, 0, 64), (2, 128, 128, 64, 0, 128), (1, 128, 128, 128, 0, 128),
    (2, 64, 64, 128, 0, 256), (1, 64, 64, 256, 0, 256), (1, 32, 32, 512, 0, 512),
    (1, 16, 16, 1024, 0, 1024), (3, 32, 32, 512, 512, 512), (3, 128, 128, 128, 128, 128),
    (3, 256, 256, 64, 64, 64),
]
only = set(sys.argv[1:])


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def report(tag, name, us, byts, flops=None):
    s = f"{tag:28s} {name:14s} {us:8.1f}us {byts / us / 1e3:6.0f} GB/s"
    if flops:
        s += f" {flops / us / 1e6:6.1f} TF/s"
    print(s, flush=True)


for mode, h, w, c0, c1, cout in SHAPES:
    C = c0 + c1
    tag = f"m{mode} {h}x{w} {C}->{cout}"
    big = 2 if mode == 2 else 1
    src = torch.randn(N, big * h, big * w, c0, device="cuda")
    sc, sh = torch.rand(c0, device="cuda") + 0.5, torch.randn(c0, device="cuda") * 0.1
    s1 = None
    if mode == 3:
        s1 = torch.randn(N, h, w, c1, device="cuda")
        v = ops.View.concat(src, s1, torch.rand(c1, device="cuda") + 0.5, torch.randn(c1, device="cuda") * 0.1)
    elif mode == 2:
        v = ops.View.pool_bnrelu(src, sc, sh)
    else:
        v = ops.View.bnrelu(src, sc, sh)
    m = N * h * w
    vin = (src.numel() + (s1.numel() if s1 is not None else 0)) * 4
    act = m * C * 4
    dk = torch.randn(3, 3, C, 1, device="cuda")
    pk = torch.randn(1, 1, C, cout, device="cuda") * 0.05
    y = torch.empty(N, h, w, C, device="cuda")
    z = torch.empty(N, h, w, cout, device="cuda")
    dz = torch.randn(N, h, w, cout, device="cuda")
    dz2 = torch.empty(N, h, w, cout, device="cuda")
    dy = torch.randn(N, h, w, C, device="cuda")
    part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
    ddk = torch.empty(3, 3, C, 1, device="cuda")
    dpk = torch.empty(1, 1, C, cout, device="cuda")
    gf = 2.0 * m * C * cout
    report(tag, "dw_fwd", timeit(lambda: ops.dwconv3x3_fwd(v, N, h, w, dk, y)), vin + act)
    report(tag, "pw_fwd", timeit(lambda: ops.pointwise_fwd(y, m, C, cout, pk, z, part)), act + m * cout * 4, gf)
    report(tag, "pw_dgrad", timeit(lambda: ops.pointwise_bwd_data(dz, m, C, cout, pk, dy)), act + m * cout * 4, gf)
    report(tag, "pw_wgrad", timeit(lambda: ops.pointwise_bwd_filter(y, dz, m, C, cout, dpk)), act + m * cout * 4, gf)
    report(tag, "dw_bwd_filter", timeit(lambda: ops.dwconv3x3_bwd_filter(v, N, h, w, dy, ddk)), vin + act)
    if mode != 2:
        dx0 = torch.empty(N, h, w, c0, device="cuda")
        dx1 = torch.empty(N, h, w, c1, device="cuda") if mode == 3 else None
        report(tag, "dw_bwd_data", timeit(lambda: ops.dwconv3x3_bwd_data(v, N, h, w, dk, dy, dx0, dx1)), 2 * act)
    coef = torch.randn(3 * cout, device="cuda") * 0.01
    scl2, shf2 = torch.rand(cout, device="cuda") + 0.5, torch.randn(cout, device="cuda") * 0.1
    report(tag, "pw_dgrad_bn", timeit(lambda: ops.pointwise_bwd_data_bnrelu(dz, z, m, C, cout, pk, scl2, shf2, coef, 0.0,
                                                                         0, dy, dz2)),
           4.0 * (2 * m * cout + m * C + m * cout), gf)
    g = torch.rand(cout, device="cuda") + 0.5
    b = torch.randn(cout, device="cuda")
    mu, rs, scl, shf = (torch.rand(cout, device="cuda") for _ in range(4))
    dg, db = torch.empty(cout, device="cuda"), torch.empty(cout, device="cuda")
    dzz = torch.empty_like(z)
    report(tag, "bn_relu_bwd", timeit(lambda: ops.bn_relu_bwd(dz, z, m, cout, mu, rs, scl, shf, True, 0.0, 0, dg, db,
                                                               dzz)), 3 * m * cout * 4)
    del src, s1, y, z, dz, dy, dzz, dz2
    torch.cuda.empty_cache()
