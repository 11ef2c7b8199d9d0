// Streaming-kernel lab: BN-backward statistics reduce (product kernel from bn.hip) vs a plain
// two-tensor read of the same bytes, at the U-Net's level-0..2 shapes.
#include "bn.hip"
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace unet;
template <class F> static double timeit(F f, int it = 20) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a)); for (int i = 0; i < it; ++i) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); CK(hipGetLastError());
    return ms * 1e3 / it;
}
// plain read of two tensors, float4 per thread, grid-stride, sum to one float per block
__global__ __launch_bounds__(256) void read2(const float4* a, const float4* b, int64_t n4, float* out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 x = a[i], y = b[i];
        s += x.x + x.y + x.z + x.w + y.x + y.y + y.z + y.w;
    }
    if (s == 123.456f) out[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void read2u(const float4* a, const float4* b, int64_t n4, float* out) {
    float s = 0.f;
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        float4 x[4], y[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { x[u] = a[i + u * stride]; y[u] = b[i + u * stride]; }
#pragma unroll
        for (int u = 0; u < 4; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w + y[u].x + y[u].y + y[u].z + y[u].w;
    }
    for (; i < n4; i += stride) { float4 x = a[i], y = b[i]; s += x.x + x.y + x.z + x.w + y.x + y.y + y.z + y.w; }
    if (s == 123.456f) out[blockIdx.x] = s;
}
int main() {
    struct S { int64_t M; int C; };
    std::vector<S> shapes = {{1048576, 64}, {1048576, 128}, {262144, 128}, {65536, 256}, {16384, 512}};
    for (auto s : shapes) {
        const int64_t n = s.M * s.C;
        float *da, *z, *out, *mean, *rstd, *sc, *sh, *part;
        CK(hipMalloc(&da, n * 4)); CK(hipMalloc(&z, n * 4)); CK(hipMalloc(&out, 1 << 20));
        CK(hipMemset(da, 0, n * 4)); CK(hipMemset(z, 0, n * 4));
        CK(hipMalloc(&mean, s.C * 4)); CK(hipMalloc(&rstd, s.C * 4)); CK(hipMalloc(&sc, s.C * 4)); CK(hipMalloc(&sh, s.C * 4));
        CK(hipMemset(mean, 0, s.C * 4)); CK(hipMemset(rstd, 0, s.C * 4)); CK(hipMemset(sc, 0, s.C * 4)); CK(hipMemset(sh, 0, s.C * 4));
        const size_t ws = unet_bn_relu_bwd_workspace(s.M, s.C);
        CK(hipMalloc(&part, ws));
        float *dg, *db, *coef; CK(hipMalloc(&dg, s.C * 4)); CK(hipMalloc(&db, s.C * 4)); CK(hipMalloc(&coef, 3 * s.C * 4));
        const double bytes = 2.0 * n * 4;
        printf("M=%ld C=%d (%.0f MB read)\n", (long)s.M, s.C, bytes / 1e6);
        for (int g : {1024, 2048, 4096}) {
            double us = timeit([&] { read2<<<g, 256>>>((float4*)da, (float4*)z, n / 4, out); });
            printf("  read2 grid %5d       %8.1f us %7.0f GB/s\n", g, us, bytes / us * 1e-3);
            us = timeit([&] { read2u<<<g, 256>>>((float4*)da, (float4*)z, n / 4, out); });
            printf("  read2u grid %5d      %8.1f us %7.0f GB/s\n", g, us, bytes / us * 1e-3);
        }
        for (float rate : {0.f, 0.2f}) {
            double us = timeit([&] { unet_bn_relu_bwd_stats(da, z, s.M, s.C, mean, rstd, sc, sh, 1, rate, 7, dg, db, coef, part, ws, 0); });
            printf("  bn_relu_bwd_stats drop %.1f %8.1f us %7.0f GB/s\n", rate, us, bytes / us * 1e-3);
        }
        CK(hipFree(da)); CK(hipFree(z)); CK(hipFree(out)); CK(hipFree(part));
        fflush(stdout);
    }
}
