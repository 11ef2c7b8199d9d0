// Activation views (see unet_view in include/unet_hip.h): read the logical input of a
// layer from raw producer outputs, applying BN affine + ReLU, 2x2 max-pool, channel
// concat and dropout on load, so the activation tensors never round-trip HBM.
#pragma once
#include "common.h"

namespace unet {

struct DView {
    const float* src0;
    const float* sc0;
    const float* sh0;
    const float* src1;
    const float* sc1;
    const float* sh1;
    int c0, c1, C;
    float rate, inv_keep;
    uint64_t seed;
};

inline DView make_dview(const unet_view& v) {
    DView d;
    d.src0 = v.src0;
    d.sc0 = v.scale0;
    d.sh0 = v.shift0;
    d.src1 = v.src1;
    d.sc1 = v.scale1;
    d.sh1 = v.shift1;
    d.c0 = v.c0;
    d.c1 = v.mode == UNET_VIEW_CONCAT ? v.c1 : 0;
    d.C = d.c0 + d.c1;
    d.rate = v.drop_rate;
    d.inv_keep = v.drop_rate > 0.f ? 1.0f / (1.0f - v.drop_rate) : 1.0f;
    d.seed = v.drop_seed;
    return d;
}

// Validates a view for an op whose logical input is (n, h, w, C).  Returns 0 or -1.
int check_view(const unet_view* v, const char* op, bool need_vec4 = false);

// Logical element loads.  (n,h,w) are logical coordinates, H/W the logical dims.
// Dropout is not applied here: callers apply drop_mult on the logical linear index.
template <int MODE>
__device__ __forceinline__ float4 view_load4(const DView& v, int n, int h, int w, int H, int W, int c) {
    if constexpr (MODE == UNET_VIEW_PLAIN) {
        return ld4(v.src0 + ((int64_t)(n * H + h) * W + w) * v.c0 + c);
    } else if constexpr (MODE == UNET_VIEW_BNRELU) {
        float4 x = ld4(v.src0 + ((int64_t)(n * H + h) * W + w) * v.c0 + c);
        return bnrelu4(x, ld4(v.sc0 + c), ld4(v.sh0 + c));
    } else if constexpr (MODE == UNET_VIEW_POOL_BNRELU) {
        const int W2 = 2 * W;
        const float* b = v.src0 + ((int64_t)(n * 2 * H + 2 * h) * W2 + 2 * w) * v.c0 + c;
        float4 sc = ld4(v.sc0 + c), sh = ld4(v.sh0 + c);
        float4 m = fma4(ld4(b), sc, sh);
        m = max4(m, fma4(ld4(b + v.c0), sc, sh));
        m = max4(m, fma4(ld4(b + (int64_t)W2 * v.c0), sc, sh));
        m = max4(m, fma4(ld4(b + (int64_t)W2 * v.c0 + v.c0), sc, sh));
        return relu4(m);
    } else {  // CONCAT: [raw upsample | bnrelu(skip)]
        const int64_t p = (int64_t)(n * H + h) * W + w;
        if (c < v.c0) return ld4(v.src0 + p * v.c0 + c);
        const int cc = c - v.c0;
        return bnrelu4(ld4(v.src1 + p * v.c1 + cc), ld4(v.sc1 + cc), ld4(v.sh1 + cc));
    }
}

template <int MODE>
__device__ __forceinline__ float view_load1(const DView& v, int n, int h, int w, int H, int W, int c) {
    if constexpr (MODE == UNET_VIEW_PLAIN) {
        return v.src0[((int64_t)(n * H + h) * W + w) * v.c0 + c];
    } else if constexpr (MODE == UNET_VIEW_BNRELU) {
        return bnrelu(v.src0[((int64_t)(n * H + h) * W + w) * v.c0 + c], v.sc0[c], v.sh0[c]);
    } else if constexpr (MODE == UNET_VIEW_POOL_BNRELU) {
        const int W2 = 2 * W;
        const float* b = v.src0 + ((int64_t)(n * 2 * H + 2 * h) * W2 + 2 * w) * v.c0 + c;
        float sc = v.sc0[c], sh = v.sh0[c];
        float m = fmaf(b[0], sc, sh);
        m = fmaxf(m, fmaf(b[v.c0], sc, sh));
        m = fmaxf(m, fmaf(b[(int64_t)W2 * v.c0], sc, sh));
        m = fmaxf(m, fmaf(b[(int64_t)W2 * v.c0 + v.c0], sc, sh));
        return relu(m);
    } else {
        const int64_t p = (int64_t)(n * H + h) * W + w;
        if (c < v.c0) return v.src0[p * v.c0 + c];
        const int cc = c - v.c0;
        return bnrelu(v.src1[p * v.c1 + cc], v.sc1[cc], v.sh1[cc]);
    }
}

// Row-indexed load for GEMM operands: row m of the (flattened) logical tensor, channels
// [c, c+4).  Only PLAIN / BNRELU (+ dropout) appear as GEMM operands.
template <int MODE, bool DROP>
__device__ __forceinline__ float4 row_load4(const DView& v, int64_t m, int c) {
    float4 x = ld4(v.src0 + m * v.c0 + c);
    if constexpr (MODE == UNET_VIEW_BNRELU) x = bnrelu4(x, ld4(v.sc0 + c), ld4(v.sh0 + c));
    if constexpr (DROP) {
        const uint64_t i = (uint64_t)m * v.C + c;
        x = mul4(x, drop_mult4(v.seed, i, v.rate, v.inv_keep));
    }
    return x;
}
template <int MODE, bool DROP>
__device__ __forceinline__ float row_load1(const DView& v, int64_t m, int c) {
    float x = v.src0[m * v.c0 + c];
    if constexpr (MODE == UNET_VIEW_BNRELU) x = bnrelu(x, v.sc0[c], v.sh0[c]);
    if constexpr (DROP) x *= drop_mult(v.seed, (uint64_t)m * v.C + c, v.rate, v.inv_keep);
    return x;
}

}  // namespace unet
