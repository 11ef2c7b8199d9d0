// "Last block finishes" within one launch: workgroups publish partial results, count their
// arrival on a per-group counter, and the workgroup that completes the count reduces the group's
// partials -- the second pass of a two-level reduction without a second launch.
//
// Visibility without an L2 writeback: on gfx950 an agent-scope release fence is `buffer_wbl2 sc1`,
// which writes back every dirty line of the XCD's L2 (all of the launch's other output).  Instead
// every value another workgroup reads is written and read as an agent-scope relaxed atomic
// (`global_store / global_load ... sc1`: coherent at the device level, so no XCD's L2 can serve a
// stale copy); the writer waits for its stores' acknowledgement (s_waitcnt vmcnt(0)) before the
// block barrier and the counter increment -- the ordering half of a release -- and the last
// arriver reads only through sc1 loads.  The finishing block resets its counter, so a counter
// array zeroed once stays ready for every later launch.
//
// Cost note (measured, r1zc/r1zd): the vmcnt(0) wait also covers the block's other stores, so in
// a streaming kernel with thousands of blocks every block lives one store round trip longer; the
// 256x256 depthwise data gradient lost 46 us per launch that way.  Use it in kernels whose blocks
// store little (the statistics reductions of bn.hip), not in the producers themselves.
#pragma once
#include "common.h"

namespace unet {

constexpr int kGroupSlabs = 64;  // slabs per first-pass block of the BN-backward statistics

// byte layout of a producer-side BN-backward partials buffer of S slabs x 2C floats:
// slabs | double chunk rows (one per 64 slabs) | cdiv(C, 64) arrival counters (u32)
inline size_t bnpart_scratch_off(int S, int C) { return align_up((size_t)S * 2 * C * sizeof(float), 256); }
inline size_t bnpart_counter_off(int S, int C) {
    return bnpart_scratch_off(S, C) + align_up((size_t)cdiv(S, kGroupSlabs) * 2 * C * sizeof(double), 256);
}
inline size_t bnpart_bytes(int S, int C) { return bnpart_counter_off(S, C) + (size_t)cdiv(C, 64) * sizeof(unsigned); }

__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// All threads of the block call this after their st_agent stores; returns true in every thread
// of the block that made `ctr` reach `expected` (and then resets it).  flag: one int of LDS.
__device__ __forceinline__ bool last_arrival(unsigned* ctr, unsigned expected, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == expected - 1;
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}

}  // namespace unet
