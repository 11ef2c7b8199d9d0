// What an in-launch "last block finishes" costs at the end of a store-heavy, one-round producer
// (the round-5 in-producer BatchNorm finish was 25-67 us slower per launch, profiles/
// r5f_fin_in_launch_ab.txt).  512 blocks x 256 threads (2 per CU, one round) each store 256 KB
// (128 MB), then per mode:
//   0 nothing more                       3 + the last block: 64 x 64 agent-scope float2 loads,
//   1 + s_waitcnt vmcnt(0) + barrier          a double row stored, a second counter (2-level)
//   2 + one agent atomic per block +     4 as 3 with plain (non-agent) loads in the last block
//       barrier (flag through LDS)       5 as 1 but the wait only in wave 0
// Launch time from HIP events over 20 back-to-back launches, minus nothing (compare rows).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int MODE>
__global__ __launch_bounds__(256, 2) void produce(float4* __restrict__ dst, size_t per_block, float2* part,
                                                  unsigned* cnt, double* out) {
    __shared__ int flag;
    __shared__ double red[256];
    float4* p = dst + blockIdx.x * per_block;
    for (size_t i = threadIdx.x; i < per_block; i += 256) p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
    if (threadIdx.x < 64) {
        const float2 v = make_float2((float)blockIdx.x, (float)threadIdx.x);
        __hip_atomic_store(reinterpret_cast<uint64_t*>(part + blockIdx.x * 64 + threadIdx.x),
                           __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (MODE == 0) return;
    if constexpr (MODE == 5) {
        if (threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (MODE == 1) return;
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == gridDim.x - 1;
        if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag = last;
    }
    __syncthreads();
    if constexpr (MODE == 2) return;
    if (!flag) return;
    // the last block: 64 rows x 64 channels of partials, 4 lanes per channel, then a row out
    const int c = threadIdx.x & 63, lane = threadIdx.x >> 6;
    double s = 0.0;
    for (int b = lane; b < 512; b += 4) {
        float2 v;
        if constexpr (MODE == 3)
            v = __builtin_bit_cast(float2, __hip_atomic_load(reinterpret_cast<uint64_t*>(part + b * 64 + c),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        else
            v = part[b * 64 + c];
        s += (double)v.x + (double)v.y;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (lane == 0) out[c] = red[c] + red[64 + c] + red[128 + c] + red[192 + c];
}

template <int MODE>
static float timeit(float4* buf, size_t per_block, float2* part, unsigned* cnt, double* out) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) produce<MODE><<<512, 256>>>(buf, per_block, part, cnt, out);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) produce<MODE><<<512, 256>>>(buf, per_block, part, cnt, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

int main() {
    const size_t bytes = (size_t)128 << 20;
    const size_t per_block = bytes / 16 / 512;
    float4* buf;
    float2* part;
    unsigned* cnt;
    double* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&part, 512 * 64 * sizeof(float2)));
    CK(hipMalloc(&cnt, 256));
    CK(hipMalloc(&out, 64 * sizeof(double)));
    CK(hipMemset(cnt, 0, 256));
    for (int rep = 0; rep < 2; ++rep) {
        printf("0 plain producer (128 MB, 512 blocks)        %7.1f us\n", timeit<0>(buf, per_block, part, cnt, out));
        printf("1 + vmcnt(0) + barrier                       %7.1f us\n", timeit<1>(buf, per_block, part, cnt, out));
        printf("5 + vmcnt(0) in wave 0 only + barrier        %7.1f us\n", timeit<5>(buf, per_block, part, cnt, out));
        printf("2 + agent atomic per block + barrier         %7.1f us\n", timeit<2>(buf, per_block, part, cnt, out));
        printf("3 + last block: 512x64 agent loads, row out  %7.1f us\n", timeit<3>(buf, per_block, part, cnt, out));
        printf("4 + last block: same with plain loads        %7.1f us\n", timeit<4>(buf, per_block, part, cnt, out));
    }
    return 0;
}
