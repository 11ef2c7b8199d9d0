// HBM streaming calibration on gfx950: the read-only, store-only and mixed
// read/write rates a 256-thread streaming kernel reaches with >= 8 waves per CU, for the two store
// shapes the U-Net epilogues use -- one dword per lane (256 contiguous bytes per wave instruction)
// and one float4 per lane (1 KiB per wave instruction) -- and for the encoder blocks' write-heavy mix
// (enc2_block1 at batch 32: 190 MB read, 425 MB written, profiles/r3e_pmc_enc2_block1.json).  Every
// byte is touched once per pass over 1.5 GiB buffers (beyond the 256 MiB Infinity Cache).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// R reads and W writes per "unit" of 16 B (VEC=4) or 4 B (VEC=1) per lane; grid-stride over n units
template <int VEC, int R, int W>
__global__ __launch_bounds__(256) void stream_k(const float* __restrict__ src, float* __restrict__ dst, size_t n,
                                                float* sink) {
    const size_t stride = (size_t)gridDim.x * 256;
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        if constexpr (VEC == 4) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float4 u = reinterpret_cast<const float4*>(src)[i + (size_t)r * n];
                v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
            }
#pragma unroll
            for (int w = 0; w < W; ++w)
                reinterpret_cast<float4*>(dst)[i + (size_t)w * n] = make_float4(v.x + w, v.y, v.z, v.w + (float)i);
            acc += v.x;
        } else {
            float v = 0.f;
#pragma unroll
            for (int r = 0; r < R; ++r) v += src[i + (size_t)r * n];
#pragma unroll
            for (int w = 0; w < W; ++w) dst[i + (size_t)w * n] = v + (float)(w + i);
            acc += v;
        }
    }
    if (acc == 1234.5f) *sink = acc;  // keeps the reads live
}

template <int VEC, int R, int W>
static void run(const char* name, float* src, float* dst, float* sink, size_t bytes_budget, int blocks_per_cu) {
    const size_t unit = VEC * 4;
    const size_t n = bytes_budget / unit / (R > W ? (R > 0 ? R : 1) : (W > 0 ? W : 1));  // units per stream
    const int blocks = 256 * blocks_per_cu;
    for (int w = 0; w < 3; ++w) stream_k<VEC, R, W><<<blocks, 256>>>(src, dst, n, sink);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int reps = 10;
    CK(hipEventRecord(a));
    for (int w = 0; w < reps; ++w) stream_k<VEC, R, W><<<blocks, 256>>>(src, dst, n, sink);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    const double by = (double)n * unit * (R + W);
    const double s = ms * 1e-3 / reps;
    printf("%-46s %2d blk/CU (%2d waves/CU): %7.1f us  %.2f TB/s  (read %.0f MB, write %.0f MB)\n", name, blocks_per_cu,
           4 * blocks_per_cu, s * 1e6, by / s * 1e-12, (double)n * unit * R / 1e6, (double)n * unit * W / 1e6);
}

int main() {
    const size_t bytes = (size_t)3 << 29;  // 1.5 GiB per buffer
    float *src, *dst, *sink;
    CK(hipMalloc(&src, bytes)); CK(hipMalloc(&dst, bytes)); CK(hipMalloc(&sink, 4));
    CK(hipMemset(src, 0x41, bytes)); CK(hipMemset(dst, 0x3f, bytes));
    for (int bpc : {2, 4, 8}) {
        run<4, 1, 0>("read-only, float4 loads", src, dst, sink, bytes, bpc);
        run<4, 0, 1>("store-only, float4 (1 KiB per wave store)", src, dst, sink, bytes, bpc);
        run<1, 0, 1>("store-only, dword (256 B per wave store)", src, dst, sink, bytes, bpc);
        run<4, 1, 1>("copy 1:1, float4", src, dst, sink, bytes, bpc);
        run<4, 1, 2>("mix 1 read : 2 writes, float4 (enc2_block1)", src, dst, sink, bytes, bpc);
        run<1, 1, 2>("mix 1 read : 2 writes, dword", src, dst, sink, bytes, bpc);
        run<4, 2, 1>("mix 2 reads : 1 write, float4", src, dst, sink, bytes, bpc);
    }
    return 0;
}
