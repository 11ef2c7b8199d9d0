// Kernel-boundary cost vs store type on gfx950: a producer writes `bytes` of float4 (plain stores, or
// __builtin_nontemporal_store), then (a) a one-block kernel, or (b) a consumer that reads it all.
// The end-of-kernel release writes the XCD L2s' dirty lines back; streaming stores should leave
// less of them, at the price of whatever the consumer loses in L2 / Infinity Cache hits.
// Timed with HIP events over 20 back-to-back pairs (the pair's time minus the producer alone).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void produce(float4* __restrict__ dst, size_t n, float v) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const float4 x = make_float4(v, v + 1.f, v + 2.f, (float)i);
        if constexpr (NT) {
            __builtin_nontemporal_store(x.x, &dst[i].x);
            __builtin_nontemporal_store(x.y, &dst[i].y);
            __builtin_nontemporal_store(x.z, &dst[i].z);
            __builtin_nontemporal_store(x.w, &dst[i].w);
        } else {
            dst[i] = x;
        }
    }
}

__global__ void tiny(float* p) {
    if (threadIdx.x == 0) p[0] += 1.f;
}

__global__ __launch_bounds__(256) void consume(const float4* __restrict__ src, size_t n, float* sink) {
    const size_t stride = (size_t)gridDim.x * 256;
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const float4 x = src[i];
        acc += x.x + x.w;
    }
    if (acc == 1234.5f) *sink = acc;
}

static float timeit(int mode, bool nt, float4* buf, size_t n, float* small, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto one = [&]() {
        if (nt) produce<true><<<2048, 256>>>(buf, n, 1.f);
        else produce<false><<<2048, 256>>>(buf, n, 1.f);
        if (mode == 1) tiny<<<1, 64>>>(small);
        if (mode == 2) consume<<<2048, 256>>>(buf, n, small);
    };
    for (int i = 0; i < 3; ++i) one();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) one();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

int main() {
    float* small;
    CK(hipMalloc(&small, 4096));
    CK(hipMemset(small, 0, 4096));
    const size_t sizes[] = {(size_t)8 << 20, (size_t)32 << 20, (size_t)128 << 20, (size_t)512 << 20};
    float4* buf;
    CK(hipMalloc(&buf, sizes[3]));
    for (size_t bytes : sizes) {
        const size_t n = bytes / 16;
        for (int nt = 0; nt < 2; ++nt) {
            const float p = timeit(0, nt, buf, n, small, 20);
            const float pt = timeit(1, nt, buf, n, small, 20);
            const float pc = timeit(2, nt, buf, n, small, 20);
            printf("%4zu MB %-13s producer %8.1f us | + tiny kernel %+7.1f us | + full read %8.1f us (read %.2f TB/s)\n",
                   bytes >> 20, nt ? "nontemporal" : "plain", p, pt - p, pc - p, bytes / ((pc - p) * 1e-6) / 1e12);
        }
    }
    return 0;
}
