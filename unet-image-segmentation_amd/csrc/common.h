// Shared device helpers for libunet_hip.so (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/unet_hip.h"

namespace unet {

// ---------------------------------------------------------------- errors ----
void set_error(const char* fmt, ...);

#define UNET_CHECK_ARG(cond, ...)        \
    do {                                 \
        if (!(cond)) {                   \
            ::unet::set_error(__VA_ARGS__); \
            return -1;                   \
        }                                \
    } while (0)

#define UNET_CHECK_LAUNCH(what)                                          \
    do {                                                                 \
        hipError_t e_ = hipGetLastError();                               \
        if (e_ != hipSuccess) {                                          \
            ::unet::set_error("%s: %s", what, hipGetErrorString(e_));     \
            return (int)e_;                                              \
        }                                                                \
    } while (0)

inline hipStream_t as_stream(unet_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Tuning knobs read from the environment exist only in the lab build (`make lab` ->
// libunet_hip_lab.so, -DUNET_LAB_BUILD, loaded by the tools through UNET_HIP_LIB).  The product
// library reads no environment: every call's behaviour is a function of its arguments.
#ifdef UNET_LAB_BUILD
int lab_knob(const char* name, int dflt);  // runtime.hip
#else
inline int lab_knob(const char*, int dflt) { return dflt; }
#endif

// -------------------------------------------------------------- vectors ----
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// pointer types __builtin_amdgcn_global_load_lds takes (global source, LDS destination)
typedef __attribute__((address_space(1))) const void gbl_void;
typedef __attribute__((address_space(3))) void lds_void;

// ------------------------------------------------ fp32 as three bf16 (split-precision GEMMs) ----
// x == hi + mid + lo EXACTLY for every finite normal fp32 x: hi = RNE_bf16(x), mid = RNE_bf16(x - hi),
// lo = x - hi - mid (both differences are exact in fp32 and lo has at most 8 significant bits).
// A GEMM then sums the six products hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid on the bf16
// MFMA (each product exact in its fp32 accumulator); the dropped mid.lo, lo.mid, lo.lo terms are
// ~2^-23 of |a b|, below the fp32 accumulation's own rounding.  See DESIGN.md "bf16x6".
typedef short bf16x8 __attribute__((ext_vector_type(8)));  // a 32x32x16 bf16 MFMA operand (4 VGPRs)
__device__ __forceinline__ unsigned bf16_bits(float x) {
    return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)x);
}
__device__ __forceinline__ float bf16_val(unsigned b) { return __uint_as_float(b << 16); }
struct Split4 {
    uint2 h, m, l;  // 4 bf16 each, element j in bits 16 (j & 1) of word j >> 1
};
__device__ __forceinline__ Split4 split4(float4 v) {
    const float x[4] = {v.x, v.y, v.z, v.w};
    unsigned h[4], m[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        h[j] = bf16_bits(x[j]);
        const float r = x[j] - bf16_val(h[j]);
        m[j] = bf16_bits(r);
        l[j] = bf16_bits(r - bf16_val(m[j]));
    }
    Split4 s;
    s.h = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    s.m = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
    s.l = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
    return s;
}
// acc += a.b over the six significant products of the split operands (a[0..2] = hi, mid, lo)
__device__ __forceinline__ floatx16 mfma_x6(const bf16x8* a, const bf16x8* b, floatx16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
    return acc;
}

// Wave issue priority of the critical-path (main-stream) backward kernels: while the weight
// gradients run beside them on a second stream, their waves win the SIMD's instruction
// arbitration (s_setprio; 0 = equal priority).  Build-time choice (UNET_MAIN_PRIO); 3 measured
// +0.7-1.0 % img/s against 0 (round 2, tools/gpu_x1.sh / gpu_x2.sh A/B on one box).
#ifndef UNET_MAIN_PRIO
#define UNET_MAIN_PRIO 3
#endif
__device__ __forceinline__ void main_stream_prio() {
    if constexpr (UNET_MAIN_PRIO > 0) __builtin_amdgcn_s_setprio(UNET_MAIN_PRIO);
}
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 mul4(float4 a, float4 b) {
    return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float4 fma4(float4 a, float4 b, float4 c) {
    return make_float4(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z),
                       fmaf(a.w, b.w, c.w));
}
__device__ __forceinline__ float4 max4(float4 a, float4 b) {
    return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
}
__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }
__device__ __forceinline__ float4 relu4(float4 v) {
    return make_float4(relu(v.x), relu(v.y), relu(v.z), relu(v.w));
}
// BatchNorm affine + ReLU as tf.nn.batch_normalization folds it: x*inv + (beta - mean*inv)
__device__ __forceinline__ float bnrelu(float x, float sc, float sh) { return relu(fmaf(x, sc, sh)); }
__device__ __forceinline__ float4 bnrelu4(float4 x, float4 sc, float4 sh) { return relu4(fma4(x, sc, sh)); }

// --------------------------------------------------------------- dropout ----
// Counter-based Bernoulli draw for the logical linear NHWC index i of an element: one splitmix64
// per group of four consecutive elements, h = splitmix64(seed + (i >> 2) * golden); element i
// takes the 16 bits (h >> 16 (i & 3)) & 0xffff, u = bits / 2^16, keep iff u >= rate.  A float4
// of channels c..c+3 (c % 4 == 0, C % 4 == 0) costs one hash.  The oracle restates this
// bit-for-bit (oracle/keras_ops.py: dropout_mult).
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t drop_hash(uint64_t seed, uint64_t group) {
    return splitmix64(seed + group * 0x9E3779B97F4A7C15ull);
}
__device__ __forceinline__ float drop_bit(uint64_t h, int lane, float rate, float inv_keep) {
    const float u = (float)((uint32_t)(h >> (16 * lane)) & 0xFFFFu) * (1.0f / 65536.0f);
    return u >= rate ? inv_keep : 0.f;
}
__device__ __forceinline__ float drop_mult(uint64_t seed, uint64_t idx, float rate, float inv_keep) {
    return drop_bit(drop_hash(seed, idx >> 2), (int)(idx & 3), rate, inv_keep);
}
// multipliers of elements idx .. idx+3, idx % 4 == 0
__device__ __forceinline__ float4 drop_mult4(uint64_t seed, uint64_t idx, float rate, float inv_keep) {
    const uint64_t h = drop_hash(seed, idx >> 2);
    return make_float4(drop_bit(h, 0, rate, inv_keep), drop_bit(h, 1, rate, inv_keep), drop_bit(h, 2, rate, inv_keep),
                       drop_bit(h, 3, rate, inv_keep));
}

// ------------------------------------------------------------ reductions ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Chan et al. parallel combination of (count, mean, M2) in double.
struct Moments {
    double n, mean, m2;
};
__device__ __forceinline__ Moments moments_combine(Moments a, Moments b) {
    if (b.n == 0.0) return a;
    if (a.n == 0.0) return b;
    double n = a.n + b.n;
    double d = b.mean - a.mean;
    Moments r;
    r.n = n;
    r.mean = a.mean + d * (b.n / n);
    r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / n);
    return r;
}

// ------------------------------------------------------------- host side ----
// Deterministic ordered reduction of S slabs of L floats: out[l] = sum_s part[s*L + l]
// (double accumulation, fixed order).  out has row stride ld_out for rows of `row`
// floats (row == L, ld_out == L for a flat copy).  part is scratch: long, narrow reductions
// sum chunks of slabs in place first (two fixed-order levels).
int reduce_slabs(float* part, int S, int64_t L, float* out, int64_t row, int64_t ld_out, hipStream_t stream);
// Two independent flat reductions over the same S slabs (one weight-gradient pass's two
// partial arrays: pointwise + depthwise kernel, head kernel + bias) in ONE launch; outputs flat.
int reduce_slabs_pair(const float* part_a, int64_t la, float* out_a, const float* part_b, int64_t lb, float* out_b,
                      int S, hipStream_t stream);

}  // namespace unet
