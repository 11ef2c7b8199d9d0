// keras.optimizers.AdamW (scripts/train.py:59,226), Keras 3 semantics:
//   weight decay first, on every trainable variable:  p -= p * wd * lr
//   m += (g - m)(1 - b1);  v += (g^2 - v)(1 - b2)
//   p -= m * alpha / (sqrt(v) + eps),  alpha = lr * sqrt(1 - b2^t) / (1 - b1^t)
// (epsilon is added to the un-corrected sqrt(v): not torch.optim.AdamW).  One fused
// multi-tensor pass over the flat parameter / gradient / moment buffers; HBM-bound
// (16 B read + 12 B written per parameter).  grad_scale folds the data-parallel 1/world.
#include "common.h"

namespace unet {
namespace {

__device__ __forceinline__ void adamw1(float& p, float g, float& m, float& v, float lr_wd, float b1c, float b2c,
                                       float eps, float alpha) {
    p = p - p * lr_wd;
    m = m + (g - m) * b1c;
    v = v + (g * g - v) * b2c;
    p = p - (m * alpha) / (sqrtf(v) + eps);
}

__global__ __launch_bounds__(256) void adamw_vec_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                        float4* __restrict__ m, float4* __restrict__ v, int64_t n4,
                                                        float lr_wd, float b1c, float b2c, float eps, float alpha,
                                                        float gs) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
        adamw1(pp.x, gg.x * gs, mm.x, vv.x, lr_wd, b1c, b2c, eps, alpha);
        adamw1(pp.y, gg.y * gs, mm.y, vv.y, lr_wd, b1c, b2c, eps, alpha);
        adamw1(pp.z, gg.z * gs, mm.z, vv.z, lr_wd, b1c, b2c, eps, alpha);
        adamw1(pp.w, gg.w * gs, mm.w, vv.w, lr_wd, b1c, b2c, eps, alpha);
        p[i] = pp;
        m[i] = mm;
        v[i] = vv;
    }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    float lr_wd, float b1c, float b2c, float eps, float alpha,
                                                    float gs) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        adamw1(p[i], g[i] * gs, m[i], v[i], lr_wd, b1c, b2c, eps, alpha);
}

}  // namespace
}  // namespace unet

using namespace unet;

extern "C" int unet_adamw_step(float* param, const float* grad, float* m, float* v, int64_t count, float lr,
                               float weight_decay, float beta1, float beta2, float eps, float alpha,
                               float grad_scale, unet_stream_t stream) {
    UNET_CHECK_ARG(param && grad && m && v && count >= 0, "unet_adamw_step: bad args");
    if (count == 0) return 0;
    hipStream_t st = as_stream(stream);
    const float lr_wd = lr * weight_decay;
    const float b1c = 1.0f - beta1, b2c = 1.0f - beta2;
    const bool vec = count % 4 == 0 && ((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0;
    if (vec) {
        const int64_t n4 = count / 4;
        int64_t grid = cdiv(n4, 256);
        if (grid > 4096) grid = 4096;
        adamw_vec_kernel<<<(unsigned)grid, 256, 0, st>>>((float4*)param, (const float4*)grad, (float4*)m, (float4*)v,
                                                         n4, lr_wd, b1c, b2c, eps, alpha, grad_scale);
    } else {
        int64_t grid = cdiv(count, 256);
        if (grid > 4096) grid = 4096;
        adamw_kernel<<<(unsigned)grid, 256, 0, st>>>(param, grad, m, v, count, lr_wd, b1c, b2c, eps, alpha,
                                                     grad_scale);
    }
    UNET_CHECK_LAUNCH("unet_adamw_step");
    return 0;
}
