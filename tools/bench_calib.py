"""Calibration: torch (hipBLASLt/rocBLAS) fp32 GEMM rates on the U-Net's pointwise shapes and
the achievable HBM copy rate, to set realistic targets for the hand-written kernels."""
import torch

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

torch.backends.cuda.matmul.allow_tf32 = False
for m, k, n in [(1048576, 64, 64), (262144, 128, 128), (65536, 256, 256), (16384, 512, 512), (4096, 1024, 1024),
                (16384, 1024, 512), (262144, 256, 128), (1048576, 128, 64), (65536, 128, 1024), (4096, 1024, 2048)]:
    a = torch.randn(m, k, device="cuda")
    b = torch.randn(k, n, device="cuda")
    c = torch.empty(m, n, device="cuda")
    us = timeit(lambda: torch.mm(a, b, out=c))
    # weight-gradient shape: (k x m) @ (m x n)
    g = torch.empty(k, n, device="cuda")
    usw = timeit(lambda: torch.mm(a.t(), c, out=g))
    print(f"mm {m}x{k}x{n}: {us:8.1f}us {2 * m * k * n / us / 1e6:6.1f} TF/s   wgrad {usw:8.1f}us "
          f"{2 * m * k * n / usw / 1e6:6.1f} TF/s", flush=True)
for mb in (64, 268, 1024):
    x = torch.empty(mb * 2 ** 20 // 4, device="cuda")
    y = torch.empty_like(x)
    us = timeit(lambda: y.copy_(x))
    print(f"copy {mb} MiB: {us:8.1f}us {2 * x.numel() * 4 / us / 1e3:6.0f} GB/s", flush=True)
