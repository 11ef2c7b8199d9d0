// FP32 MFMA ceiling under load on gfx950 (VERDICT r4 item 2 calibration): what a 256-thread,
// 2-blocks-per-CU kernel shaped like the rows GEMM (4 waves x 2x2 32x32 tiles) sustains when its
// v_mfma_f32_32x32x2_f32 stream is fed (a) from registers, (b) from LDS (ds_read_b128 fragments, one
// barrier per 16-deep stage), (c) as (b) plus a streaming global read per stage, (d) as (c) plus
// the stage's LDS writes.  Each block stamps s_memtime / s_memrealtime at its start and end, so the
// in-kernel clock (cycles / (realtime ticks / 100 MHz)) is printed beside TF/s: it separates a
// throttled clock (DVFS) from idle matrix-pipe cycles.  Random operands (not zeros: zeros clock up).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void mfma_k(const float* __restrict__ src, float* out, int iters,
                                              unsigned long long* stamps) {
    __shared__ __attribute__((aligned(16))) float L[2][128 * 36 * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    unsigned long long t0 = 0, r0 = 0;
    if (tid == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = tid; i < 2 * 128 * 36 * 2; i += 256) (&L[0][0])[i] = src[(blockIdx.x * 7919 + i) & 0xFFFFF];
    __syncthreads();
    floatx16 acc[2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    float4 fa[2], fb[2];
    for (int t = 0; t < 2; ++t) {
        fa[t] = *reinterpret_cast<const float4*>(&L[0][((wave >> 1) * 64 + t * 32 + lo) * 36 + 4 * hi]);
        fb[t] = *reinterpret_cast<const float4*>(&L[0][128 * 36 + ((wave & 1) * 64 + t * 32 + lo) * 36 + 4 * hi]);
    }
    const float* gp = src + ((size_t)blockIdx.x * 256 + tid) * 4;
    float4 g4 = make_float4(0, 0, 0, 0);
    for (int it = 0; it < iters; ++it) {
        const int buf = it & 1;
        if constexpr (MODE >= 2) {  // a streaming read per stage (128 rows x 16 k x 2 operands = 16 KB/block)
            const float4 v = *reinterpret_cast<const float4*>(gp + (((size_t)it * 1024 * 256 * 4) & ((1u << 26) - 1)));
            g4.x += v.x; g4.y += v.y; g4.z += v.z; g4.w += v.w;
            if constexpr (MODE >= 3) *reinterpret_cast<float4*>(&L[buf ^ 1][tid * 4 + 4096]) = v;
        }
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
            if constexpr (MODE >= 1) {
                for (int t = 0; t < 2; ++t) {
                    fa[t] = *reinterpret_cast<const float4*>(&L[buf][((wave >> 1) * 64 + t * 32 + lo) * 36 + kg * 8 + 4 * hi]);
                    fb[t] = *reinterpret_cast<const float4*>(&L[buf][128 * 36 + ((wave & 1) * 64 + t * 32 + lo) * 36 + kg * 8 + 4 * hi]);
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].x, fb[b].x, acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].y, fb[b].y, acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].z, fb[b].z, acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].w, fb[b].w, acc[a][b], 0, 0, 0);
                }
        }
        if constexpr (MODE >= 4) {  // + VALU work per stage (MODE 4: 64, MODE 5: 128 independent fmaf)
            constexpr int NV = MODE == 4 ? 16 : 32;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                g4.x = fmaf(g4.x, 1.0001f, fa[0].x);
                g4.y = fmaf(g4.y, 1.0001f, fa[0].y);
                g4.z = fmaf(g4.z, 1.0001f, fa[1].x);
                g4.w = fmaf(g4.w, 1.0001f, fa[1].y);
            }
        }
        if constexpr (MODE >= 6) {  // + 8 ds_write_b128 per stage (the GEMM's A + B staging)
#pragma unroll
            for (int r = 0; r < 8; ++r) *reinterpret_cast<float4*>(&L[buf ^ 1][(tid * 4 + r * 1024) % (128 * 36 * 2 - 4)]) = g4;
        }
        if constexpr (MODE >= 1) __syncthreads();
    }
    float s = g4.x + g4.y + g4.z + g4.w;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int r = 0; r < 16; ++r) s += acc[a][b][r];
    out[blockIdx.x * 256 + tid] = s;
    if (tid == 0) {
        stamps[4 * blockIdx.x + 0] = t0;
        stamps[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memtime();
        stamps[4 * blockIdx.x + 2] = r0;
        stamps[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();
    }
}


typedef short bf16x8 __attribute__((ext_vector_type(8)));
// bf16 32x32x16 MFMA stream with NV VALU fmaf per stage (same stage structure, 12 MFMAs per stage per wave
// = 384 cycles, the bf16x6 equivalent of 2 f32 32x32x2 k-groups x 2x2 tiles costs 6 x 4 = 24 MFMAs)
template <int NV>
__global__ __launch_bounds__(256) void mfma_bf16_k(const float* __restrict__ src, float* out, int iters,
                                                   unsigned long long* stamps) {
    __shared__ __attribute__((aligned(16))) float L[2][128 * 36 * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    unsigned long long t0 = 0, r0 = 0;
    if (tid == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = tid; i < 2 * 128 * 36 * 2; i += 256) (&L[0][0])[i] = src[(blockIdx.x * 7919 + i) & 0xFFFFF];
    __syncthreads();
    floatx16 acc[2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    float4 g4 = make_float4(0, 0, 0, 0);
    for (int it = 0; it < iters; ++it) {
        const int buf = it & 1;
        bf16x8 fa[2], fb[2];
        for (int t = 0; t < 2; ++t) {
            fa[t] = *reinterpret_cast<const bf16x8*>(&L[buf][((wave >> 1) * 64 + t * 32 + lo) * 36 + 4 * hi]);
            fb[t] = *reinterpret_cast<const bf16x8*>(&L[buf][128 * 36 + ((wave & 1) * 64 + t * 32 + lo) * 36 + 4 * hi]);
        }
#pragma unroll
        for (int rep = 0; rep < 6; ++rep)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < NV / 4; ++v) {
            g4.x = fmaf(g4.x, 1.0001f, (float)fa[0][0]);
            g4.y = fmaf(g4.y, 1.0001f, (float)fa[0][1]);
            g4.z = fmaf(g4.z, 1.0001f, (float)fa[1][0]);
            g4.w = fmaf(g4.w, 1.0001f, (float)fa[1][1]);
        }
        __syncthreads();
    }
    float s = g4.x + g4.y + g4.z + g4.w;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int r = 0; r < 16; ++r) s += acc[a][b][r];
    out[blockIdx.x * 256 + tid] = s;
    if (tid == 0) {
        stamps[4 * blockIdx.x + 0] = t0;
        stamps[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memtime();
        stamps[4 * blockIdx.x + 2] = r0;
        stamps[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();
    }
}
template <int NV>
static void run_bf16(const char* name, const float* src, float* out, unsigned long long* st, int blocks, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 20; ++w) mfma_bf16_k<NV><<<blocks, 256>>>(src, out, iters, st);
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int w = 0; w < reps; ++w) mfma_bf16_k<NV><<<blocks, 256>>>(src, out, iters, st);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double mf = (double)blocks * 4 * iters * 24;  // MFMAs
    const double cyc_per_mfma = us * 1e-6 * 2.39e9 / (mf / 1024.0);  // per SIMD
    printf("%-34s %9.1f us  %.1f cycles per bf16 MFMA per SIMD (32 = back-to-back)\n", name, us, cyc_per_mfma);
}

template <int MODE>
static void run(const char* name, const float* src, float* out, unsigned long long* st, int blocks, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 20; ++w) mfma_k<MODE><<<blocks, 256>>>(src, out, iters, st);  // warm the clock up
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int w = 0; w < reps; ++w) mfma_k<MODE><<<blocks, 256>>>(src, out, iters, st);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> h(4 * blocks);
    CK(hipMemcpy(h.data(), st, 8 * 4 * blocks, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (int i = 0; i < blocks; ++i) {
        const double cyc = (double)(h[4 * i + 1] - h[4 * i]), rt = (double)(h[4 * i + 3] - h[4 * i + 2]);
        if (rt > 0) clk.push_back(cyc / rt * 0.1);  // GHz (realtime at 100 MHz)
    }
    std::sort(clk.begin(), clk.end());
    const double us = ms * 1e3 / reps;
    const double fl = (double)blocks * 4 * iters * 2 * 16 * 4096.0;  // waves x iters x kg x MFMAs x flop
    printf("%-34s %9.1f us  %7.1f TF/s  frac %.3f  in-kernel clock median %.3f GHz (min %.3f max %.3f)\n", name, us,
           fl / us * 1e-6, fl / us * 1e-6 / 157.3, clk[clk.size() / 2], clk.front(), clk.back());
}

int main() {
    const size_t n = (size_t)1 << 26;
    std::vector<float> h(n);
    srand(7);
    for (size_t i = 0; i < n; ++i) h[i] = (float)rand() / RAND_MAX - 0.5f;
    float *src, *out;
    unsigned long long* st;
    CK(hipMalloc(&src, n * 4)); CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
    const int blocks = 512;
    CK(hipMalloc(&out, blocks * 256 * 4)); CK(hipMalloc(&st, blocks * 4 * 8));
    const int iters = 2048;
    run<0>("registers only", src, out, st, blocks, iters);
    run<1>("LDS fragments + barrier", src, out, st, blocks, iters);
    run<2>("+ streaming global read", src, out, st, blocks, iters);
    run<3>("+ LDS write of it", src, out, st, blocks, iters);
    run<4>("+ 64 VALU fma / stage", src, out, st, blocks, iters);
    run<5>("+ 128 VALU fma / stage", src, out, st, blocks, iters);
    run<6>("+ 128 VALU + 8 ds_write_b128", src, out, st, blocks, iters);
    run<3>("mode 3, 32 stages (K=512 at BK16)", src, out, st, blocks, 32);
    run<6>("mode 6, 32 stages", src, out, st, blocks, 32);
    run<0>("registers only (again)", src, out, st, blocks, iters);
    run_bf16<0>("bf16 MFMA + LDS frags + barrier", src, out, st, blocks, iters);
    run_bf16<64>("bf16 + 64 VALU / stage", src, out, st, blocks, iters);
    run_bf16<128>("bf16 + 128 VALU / stage", src, out, st, blocks, iters);
    run_bf16<256>("bf16 + 256 VALU / stage", src, out, st, blocks, iters);
    return 0;
}
