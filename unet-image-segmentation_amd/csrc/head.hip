// Output layer + loss + metric kernels:
//   head      : Conv2D(num_classes, 1, activation=sigmoid|softmax)   model/u_net.py:105-112
//   dice/iou  : dice_coef / iou_coef / dice_loss / iou_loss            utils/metrics.py:6-62,
//                                                                      utils/loss.py:9-48
//   MeanIoU   : keras.metrics.MeanIoU(num_classes)                     scripts/train.py:231,
//                                                                      scripts/benchmark.py:237-277
// The head is HBM-bound (64 -> ncls per pixel).  Binary: a lane group per pixel, xor-shuffle
// dot products (head_fwd_bin_kernel); multi-class: one lane per pixel, the (Cin x ncls) kernel in
// LDS (broadcast reads).  Dice sums are per (image, class) over H*W: per-block
// partials, then one fixed-order finalize in double.
#include "view.h"

namespace unet {

int head_wgrad(const unet_view* x, int64_t M, const float* dlogit, int ncls, float* dkernel, void* ws,
               size_t ws_bytes, hipStream_t st);
size_t head_wgrad_workspace(int64_t M, int cin, int ncls);
int colsum(const float* x, int64_t rows, int cols, float* out, void* ws, size_t ws_bytes, hipStream_t st);
size_t colsum_workspace(int64_t rows, int cols);

namespace {

constexpr int kMaxCin = 256;
constexpr int kMaxCls = 32;

// Binary head, Cin = 4G (G lanes per pixel, one channel quad each): every lane issues U
// independent float4 loads (U pixels, each wave's loads contiguous 1 KB runs), applies the
// BN+ReLU view, dots with its kernel quad held in registers, and the G lanes of a pixel reduce
// with xor shuffles.  No LDS, no barriers: the loads of a wave stay in flight together.
template <int MODE, int G>
__global__ __launch_bounds__(256) void head_fwd_bin_kernel(DView v, int64_t M, const float* __restrict__ W,
                                                           const float* __restrict__ bias, float* __restrict__ prob) {
    constexpr int PPW = 64 / G;  // pixels per wave per slot
    constexpr int U = 4;
    constexpr int PB = 4 * U * PPW;  // pixels per block iteration
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane % G, ps = lane / G;
    const int c = 4 * q;
    const float4 wk = ld4(W + c);  // Keras (1, 1, Cin, 1): W[c]
    float4 sc = f4(1.f), sh = f4(0.f);
    if constexpr (MODE == UNET_VIEW_BNRELU) {
        sc = ld4(v.sc0 + c);
        sh = ld4(v.sh0 + c);
    }
    const float b = bias ? bias[0] : 0.f;
    for (int64_t base = (int64_t)blockIdx.x * PB; base < M; base += (int64_t)gridDim.x * PB) {
        const int64_t p0 = base + wave * U * PPW + ps;
        float4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t m = p0 + u * PPW;
            x[u] = m < M ? ld4(v.src0 + m * (4 * G) + c) : f4(0.f);
        }
        float s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4 a = x[u];
            if constexpr (MODE == UNET_VIEW_BNRELU) a = bnrelu4(a, sc, sh);
            s[u] = fmaf(a.x, wk.x, fmaf(a.y, wk.y, fmaf(a.z, wk.z, a.w * wk.w)));
        }
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1)
#pragma unroll
            for (int u = 0; u < U; ++u) s[u] += __shfl_xor(s[u], off, 64);
        if (q == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t m = p0 + u * PPW;
                if (m < M) prob[m] = 1.0f / (1.0f + expf(-(s[u] + b)));
            }
        }
    }
}

// Pixel tile of TP = 8192 / Cin (binary) or 4096 / Cin (multi-class) pixels: the tile's activations are staged through LDS with
// coalesced float4 loads (one lane per channel quad), then one lane per pixel forms the logits.
template <int MODE, int NC>
__global__ __launch_bounds__(256) void head_fwd_kernel(DView v, int64_t M, int ncls, const float* __restrict__ W,
                                                       const float* __restrict__ bias, float* __restrict__ prob) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int Cin = v.c0, CQ = Cin / 4, LA = Cin + 1, TP = min(256, (NC == 1 ? 8192 : 4096) / Cin);  // LDS <= 64 KB
    float* Ws = smem;                // [Cin][NC]
    float* bs = Ws + kMaxCin * NC;   // [NC]
    float* A = bs + NC;              // [TP][Cin + 1]
    for (int i = threadIdx.x; i < Cin * NC; i += 256) {
        const int k = i / NC, c = i % NC;
        Ws[i] = c < ncls ? W[k * ncls + c] : 0.f;
    }
    if (threadIdx.x < NC) bs[threadIdx.x] = (threadIdx.x < ncls && bias) ? bias[threadIdx.x] : 0.f;
    for (int64_t m0 = (int64_t)blockIdx.x * TP; m0 < M; m0 += (int64_t)gridDim.x * TP) {
        __syncthreads();
        for (int idx = threadIdx.x; idx < TP * CQ; idx += 256) {
            const int p = idx / CQ, kq = idx - (idx / CQ) * CQ;
            const int64_t m = m0 + p;
            float4 x = f4(0.f);
            if (m < M) x = row_load4<MODE, false>(v, m, 4 * kq);
            float* a = A + p * LA + 4 * kq;
            a[0] = x.x;
            a[1] = x.y;
            a[2] = x.z;
            a[3] = x.w;
        }
        __syncthreads();
        const int p = threadIdx.x;
        const int64_t m = m0 + p;
        if (p >= TP || m >= M) continue;
        float l[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) l[c] = bs[c];
        for (int k = 0; k < Cin; ++k) {
            const float a = A[p * LA + k];
#pragma unroll
            for (int c = 0; c < NC; ++c) l[c] = fmaf(a, Ws[k * NC + c], l[c]);
        }
        if (ncls == 1) {
            prob[m] = 1.0f / (1.0f + expf(-l[0]));
        } else {
            float mx = -INFINITY;
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (c < ncls) mx = fmaxf(mx, l[c]);
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                l[c] = c < ncls ? expf(l[c] - mx) : 0.f;
                s += l[c];
            }
            const float inv = 1.0f / s;
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (c < ncls) prob[m * ncls + c] = l[c] * inv;
        }
    }
}

// part[n][blk][3][ncls] = {sum t*p, sum t, sum p} over this block's pixels of image n
template <int NC>
__global__ __launch_bounds__(256) void dice_partial_kernel(const float* __restrict__ yt, const float* __restrict__ yp,
                                                           int64_t hw, int ncls, int64_t ppb,
                                                           float* __restrict__ part) {
    const int n = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
    float I[NC], T[NC], P[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) I[c] = T[c] = P[c] = 0.f;
    const int64_t p0 = (int64_t)blk * ppb;
    const int64_t p1 = p0 + ppb < hw ? p0 + ppb : hw;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
        const int64_t base = ((int64_t)n * hw + p) * ncls;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < ncls) {
                const float t = yt[base + c], q = yp[base + c];
                I[c] = fmaf(t, q, I[c]);
                T[c] += t;
                P[c] += q;
            }
        }
    }
    __shared__ float red[4][3 * NC];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const float a = wave_sum(I[c]), b = wave_sum(T[c]), d = wave_sum(P[c]);
        if (lane == 0) {
            red[wave][c] = a;
            red[wave][NC + c] = b;
            red[wave][2 * NC + c] = d;
        }
    }
    __syncthreads();
    if (threadIdx.x < 3 * NC) {
        const int j = threadIdx.x / NC, c = threadIdx.x % NC;
        if (c < ncls) {
            const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
            part[(((int64_t)n * nblk + blk) * 3 + j) * ncls + c] = s;
        }
    }
}

// Multi-class form: the block's pixel rows (ncls contiguous floats each) staged a 256-pixel tile
// at a time through LDS with coalesced loads, then lane (class c, 32-row group g) sums its column
// slice; the 8 groups are combined in a fixed order at the end.  (The one-lane-per-pixel form
// read 21-float rows lane-strided: 77 us for the batch-8 21-class sums, profiles/r4j_cfg4_trace.txt.)
template <int NC>
__global__ __launch_bounds__(256) void dice_partial_m_kernel(const float* __restrict__ yt, const float* __restrict__ yp,
                                                             int64_t hw, int ncls, int64_t ppb, float* __restrict__ part) {
    __shared__ float Ys[256 * NC], Qs[256 * NC];
    const int n = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
    const int c = threadIdx.x % NC, g = threadIdx.x / NC;
    float I = 0.f, T = 0.f, P = 0.f;
    const int64_t p0 = (int64_t)blk * ppb;
    const int64_t p1 = p0 + ppb < hw ? p0 + ppb : hw;
    for (int64_t t0 = p0; t0 < p1; t0 += 256) {
        const int np = p1 - t0 < 256 ? (int)(p1 - t0) : 256;
        const int cnt = np * ncls;
        const int64_t f0 = ((int64_t)n * hw + t0) * ncls;
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += 256) {
            Ys[i] = yt[f0 + i];
            Qs[i] = yp[f0 + i];
        }
        __syncthreads();
        if (g < 8 && c < ncls) {
            const int r1 = (g + 1) * 32 < np ? (g + 1) * 32 : np;
            for (int r = g * 32; r < r1; ++r) {
                const float y = Ys[r * ncls + c], q = Qs[r * ncls + c];
                I = fmaf(y, q, I);
                T += y;
                P += q;
            }
        }
    }
    __syncthreads();
    if (g < 8) {
        Ys[g * NC + c] = I;
        Ys[8 * NC + g * NC + c] = T;
        Ys[16 * NC + g * NC + c] = P;
    }
    __syncthreads();
    if (threadIdx.x < 3 * NC) {
        const int j = threadIdx.x / NC, cc = threadIdx.x % NC;
        if (cc < ncls) {
            float sacc = 0.f;
            for (int q = 0; q < 8; ++q) sacc += Ys[j * 8 * NC + q * NC + cc];
            part[(((int64_t)n * nblk + blk) * 3 + j) * ncls + cc] = sacc;
        }
    }
}

// Per (image, class) term: the block partials summed in double by a group of lanes and an
// xor-shuffle tree (fixed lane order); the dice / iou terms then summed by one wave in a fixed
// order -- deterministic, and no thread walks all nblk partials or all terms serially.
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__global__ __launch_bounds__(1024) void dice_finalize_kernel(const float* part, int N, int nblk, int ncls,
                                                            float smooth, float* __restrict__ sums,
                                                            float* __restrict__ result) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int kMaxTerms = 1024;  // terms kept in LDS for the ordered sum (N * ncls beyond: second pass)
    __shared__ float td[kMaxTerms], ti[kMaxTerms];
    __shared__ double acc[2];
    // all partials staged in LDS with coalesced loads when they fit: the per-term walks
    // then wait on LDS, not on a dependent global load a term
    constexpr int kStage = 34816;  // 136 KB
    __shared__ float pst[kStage];
    const int64_t total = (int64_t)N * nblk * 3 * ncls;
    if (total <= kStage) {
        // 8 independent loads in flight per thread (a load-store pair per iteration exposed the
        // load latency ~32 times: 31 us for 8 x 21-class partials)
        const int bd = blockDim.x;
        for (int i0 = threadIdx.x; i0 < (int)total; i0 += 8 * bd) {
            float t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = i0 + u * bd < (int)total ? part[i0 + u * bd] : 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (i0 + u * bd < (int)total) pst[i0 + u * bd] = t[u];
        }
        __syncthreads();
        part = pst;
    }
    if (threadIdx.x == 0) acc[0] = acc[1] = 0.0;
    // 8 lanes a term (lane g sums partials g, g + 8, ... in double, then an xor tree within the
    // group): 128 terms at a time instead of one a wave; the terms' dice / iou values are then
    // summed by one wave (lane t: terms t, t + 64, ..., then its xor tree) -- fixed orders both
    constexpr int G = 8;
    const int grp = threadIdx.x / G, gl = threadIdx.x % G, ngrp = (int)(blockDim.x / G);
    for (int base = 0; base < N * ncls; base += kMaxTerms) {
        const int nt = N * ncls - base < kMaxTerms ? N * ncls - base : kMaxTerms;
        for (int k0 = 0; k0 < nt; k0 += ngrp) {  // (uniform trip count: the shuffles see every lane)
            const int k = k0 + grp;
            const int idx = base + (k < nt ? k : 0), n = idx / ncls, c = idx % ncls;
            double I = 0.0, T = 0.0, P = 0.0;
            if (k < nt)
                for (int b = gl; b < nblk; b += G) {
                    const int64_t o = (((int64_t)n * nblk + b) * 3) * ncls + c;
                    I += part[o];
                    T += part[o + ncls];
                    P += part[o + 2 * ncls];
                }
#pragma unroll
            for (int o = G / 2; o > 0; o >>= 1) {
                I += __shfl_xor(I, o, 64);
                T += __shfl_xor(T, o, 64);
                P += __shfl_xor(P, o, 64);
            }
            if (gl == 0 && k < nt) {
                const float fi = (float)I, ft = (float)T, fp = (float)P;
                if (sums) {
                    sums[idx * 3 + 0] = fi;
                    sums[idx * 3 + 1] = ft;
                    sums[idx * 3 + 2] = fp;
                }
                td[k] = (2.0f * fi + smooth) / (ft + fp + smooth);
                ti[k] = (fi + smooth) / (ft + fp - fi + smooth);
            }
        }
        __syncthreads();
        if (wave == 0) {
            double d = 0.0, i = 0.0;
            for (int k = lane; k < nt; k += 64) {
                d += (double)td[k];
                i += (double)ti[k];
            }
            d = wave_sum_d(d);
            i = wave_sum_d(i);
            if (lane == 0) {
                acc[0] += d;
                acc[1] += i;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double cnt = (double)N * ncls;
        const float dice = (float)(acc[0] / cnt);
        result[0] = 1.0f - dice;
        result[1] = dice;
        result[2] = (float)(acc[1] / cnt);
    }
}

// d(loss)/d(prob) for one (pixel, class) from the per-(image, class) sums
template <int LOSS>
__device__ __forceinline__ float loss_grad(float t, const float* s3, float smooth, float gscale) {
    const float I = s3[0], T = s3[1], P = s3[2];
    if constexpr (LOSS == UNET_LOSS_DICE) {
        const float nm = 2.0f * I + smooth, den = T + P + smooth;
        return -gscale * (2.0f * t * den - nm) / (den * den);
    } else {
        const float j = I + smooth, u = T + P - I + smooth;
        return -gscale * (t * u - j * (1.0f - t)) / (u * u);
    }
}

// Binary head (ncls == 1), fully fused backward over 256-pixel tiles:
//   phase 1: one lane per pixel -> dlogit = dL/dp * p (1 - p) into LDS (and the db sum);
//   phase 2: one lane per (pixel, channel quad), coalesced: dx = W dlogit, and
//            dW += relu(bn(z)) * dlogit accumulated in registers across tiles;
//   end: fixed-order LDS reduction -> per-block partials of dW (Cin) and db (1).
// STATS (BNRELU view): dx is the whole da of the last decoder block, so the kernel also emits
// that block's BatchNorm-backward partial sums (bnpart[block][0][c] = sum g, [1][c] = sum g*xhat,
// g = dx*[z*sc+sh > 0], xhat = (z-mu)*rs) instead of leaving them to a pass over (dx, z).
// DLOUT (with STATS): dx = dlogit (x) W is rank one; only dlogit goes out (one float per pixel,
// `dx` is the dlogit buffer) and the consumer forms dx on load with the same product.
template <int MODE, int LOSS, bool STATS = false, bool DLOUT = false>
__global__ __launch_bounds__(256) void head_bwd1_kernel(DView v, int64_t M, int64_t hw, const float* __restrict__ W,
                                                        const float* __restrict__ prob, const float* __restrict__ yt,
                                                        const float* __restrict__ sums, float smooth, float gscale,
                                                        float* __restrict__ dx, float* __restrict__ part_w,
                                                        float* __restrict__ part_b, const float* __restrict__ mu = nullptr,
                                                        const float* __restrict__ rs = nullptr,
                                                        float* __restrict__ bnpart = nullptr) {
    main_stream_prio();
    __shared__ float dls[256];
    __shared__ float4 red[256];
    const int Cin = v.c0, CQ = Cin / 4;
    const int kq = threadIdx.x % CQ;  // CQ divides 256 (launcher checks)
    const float4 w4 = ld4(W + 4 * kq);
    float4 dw = f4(0.f);
    float db = 0.f;
    float4 s1 = f4(0.f), s2 = f4(0.f), hsc = f4(1.f), hsh = f4(0.f), smu = f4(0.f), srs = f4(0.f);
    if constexpr (STATS) {
        hsc = ld4(v.sc0 + 4 * kq);
        hsh = ld4(v.sh0 + 4 * kq);
        if (mu) {
            smu = ld4(mu + 4 * kq);
            srs = ld4(rs + 4 * kq);
        }
    }
    for (int64_t m0 = (int64_t)blockIdx.x * 256; m0 < M; m0 += (int64_t)gridDim.x * 256) {
        __syncthreads();
        {
            const int64_t m = m0 + threadIdx.x;
            float dl = 0.f;
            if (m < M) {
                const float p = prob[m];
                const float g = loss_grad<LOSS>(yt[m], sums + (m / hw) * 3, smooth, gscale);
                dl = g * p * (1.0f - p);
            }
            dls[threadIdx.x] = dl;
            if constexpr (DLOUT) {
                if (m < M) dx[m] = dl;
            }
            db += dl;
        }
        __syncthreads();
        for (int p = threadIdx.x / CQ; p < 256; p += 256 / CQ) {
            const int64_t m = m0 + p;
            if (m >= M) break;
            const float dl = dls[p];
            if constexpr (STATS) {
                const float4 zr = ld4(v.src0 + m * Cin + 4 * kq);
                const float4 a = bnrelu4(zr, hsc, hsh);
                dw = fma4(a, f4(dl), dw);
                const float4 d = mul4(w4, f4(dl));
                if constexpr (!DLOUT) st4(dx + m * Cin + 4 * kq, d);
                const float4 gm = make_float4(a.x > 0.f ? d.x : 0.f, a.y > 0.f ? d.y : 0.f, a.z > 0.f ? d.z : 0.f,
                                              a.w > 0.f ? d.w : 0.f);
                s1 = add4(s1, gm);
                const float4 xh = make_float4((zr.x - smu.x) * srs.x, (zr.y - smu.y) * srs.y, (zr.z - smu.z) * srs.z,
                                              (zr.w - smu.w) * srs.w);
                s2 = fma4(gm, xh, s2);
            } else {
                const float4 a = row_load4<MODE, false>(v, m, 4 * kq);
                dw = fma4(a, f4(dl), dw);
                st4(dx + m * Cin + 4 * kq, mul4(w4, f4(dl)));
            }
        }
    }
    if constexpr (STATS) {  // fixed-order per-channel-quad sums of the block's threads
        __syncthreads();
        red[threadIdx.x] = s1;
        __syncthreads();
        if (threadIdx.x < CQ) {
            float4 t = red[threadIdx.x];
            for (int q = threadIdx.x + CQ; q < 256; q += CQ) t = add4(t, red[q]);
            st4(bnpart + (int64_t)blockIdx.x * 2 * Cin + 4 * threadIdx.x, t);
        }
        __syncthreads();
        red[threadIdx.x] = s2;
        __syncthreads();
        if (threadIdx.x < CQ) {
            float4 t = red[threadIdx.x];
            for (int q = threadIdx.x + CQ; q < 256; q += CQ) t = add4(t, red[q]);
            st4(bnpart + (int64_t)blockIdx.x * 2 * Cin + Cin + 4 * threadIdx.x, t);
        }
    }
    __syncthreads();
    red[threadIdx.x] = dw;
    __syncthreads();
    if (threadIdx.x < CQ) {
        float4 s = red[threadIdx.x];
        for (int q = threadIdx.x + CQ; q < 256; q += CQ) s = add4(s, red[q]);
        st4(part_w + (int64_t)blockIdx.x * Cin + 4 * threadIdx.x, s);
    }
    const float dbs = wave_sum(db);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) dls[threadIdx.x >> 6] = dbs;
    __syncthreads();
    if (threadIdx.x == 0) part_b[blockIdx.x] = dls[0] + dls[1] + dls[2] + dls[3];
}

// Multi-class head: dlogit (softmax backward) to global for the weight-gradient GEMM, and dx
// written coalesced per (pixel, channel quad) from LDS copies of W and the tile's dlogits.
template <int NC, int LOSS>
__global__ __launch_bounds__(256) void head_bwd_kernel(int64_t M, int64_t hw, int Cin, int ncls,
                                                       const float* __restrict__ W, const float* __restrict__ prob,
                                                       const float* __restrict__ yt, const float* __restrict__ sums,
                                                       float smooth, float gscale, float* __restrict__ dlogit,
                                                       float* __restrict__ dx) {
    __shared__ float Ws[kMaxCin * NC];
    __shared__ float dls[256 * NC];
    for (int i = threadIdx.x; i < Cin * NC; i += 256) {
        const int k = i / NC, c = i % NC;
        Ws[i] = c < ncls ? W[k * ncls + c] : 0.f;
    }
    const int CQ = Cin / 4;
    for (int64_t m0 = (int64_t)blockIdx.x * 256; m0 < M; m0 += (int64_t)gridDim.x * 256) {
        __syncthreads();
        {
            const int64_t m = m0 + threadIdx.x;
            float p[NC], dl[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                p[c] = 0.f;
                dl[c] = 0.f;
                if (c < ncls && m < M) {
                    p[c] = prob[m * ncls + c];
                    dl[c] = loss_grad<LOSS>(yt[m * ncls + c], sums + ((m / hw) * ncls + c) * 3, smooth, gscale);
                }
            }
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) s = fmaf(dl[c], p[c], s);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                dl[c] = p[c] * (dl[c] - s);
                dls[threadIdx.x * NC + c] = dl[c];
                if (c < ncls && m < M) dlogit[m * ncls + c] = dl[c];
            }
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < 256 * CQ; idx += 256) {
            const int p = idx / CQ, kq = idx - (idx / CQ) * CQ;
            const int64_t m = m0 + p;
            if (m >= M) continue;
            float4 o = f4(0.f);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const float d = dls[p * NC + c];
                o.x = fmaf(Ws[(4 * kq + 0) * NC + c], d, o.x);
                o.y = fmaf(Ws[(4 * kq + 1) * NC + c], d, o.y);
                o.z = fmaf(Ws[(4 * kq + 2) * NC + c], d, o.z);
                o.w = fmaf(Ws[(4 * kq + 3) * NC + c], d, o.w);
            }
            st4(dx + m * Cin + 4 * kq, o);
        }
    }
}

// Multi-class head forward, one pixel per thread over 256-pixel tiles (Cin <= 64): the tile's
// activations staged through LDS with coalesced float4 loads (view applied), the kernel as
// [Cin][NC] rows read 4 classes at a time (ds_read_b128, one address per wave: broadcast), logits
// in NC registers (NC = the class count rounded up to 4), softmax, probabilities out.
// (The earlier one-float-per-class LDS reads over 32 padded classes made the 21-class head
// LDS-bound: 153 us per batch-8 forward, profiles/r4j_cfg4_trace.txt.)
template <int MODE, int NC>
__global__ __launch_bounds__(256) void head_fwdm_kernel(DView v, int64_t M, int ncls, const float* __restrict__ W,
                                                        const float* __restrict__ bias, float* __restrict__ prob) {
    constexpr int CMAX = 64, LA = CMAX + 4;
    __shared__ __attribute__((aligned(16))) float Ws[CMAX * NC];
    __shared__ __attribute__((aligned(16))) float A[256 * LA];
    const int Cin = v.c0, CQ = Cin / 4;
    for (int i = threadIdx.x; i < Cin * NC; i += 256) {
        const int k = i / NC, c = i - k * NC;
        Ws[i] = c < ncls ? W[k * ncls + c] : 0.f;
    }
    float bl[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) bl[c] = (c < ncls && bias) ? bias[c] : 0.f;
    for (int64_t m0 = (int64_t)blockIdx.x * 256; m0 < M; m0 += (int64_t)gridDim.x * 256) {
        __syncthreads();
        for (int idx = threadIdx.x; idx < 256 * CQ; idx += 256) {
            const int p = idx / CQ, kq = idx - p * CQ;
            const int64_t m = m0 + p;
            const float4 x = m < M ? row_load4<MODE, false>(v, m, 4 * kq) : f4(0.f);
            *reinterpret_cast<float4*>(&A[p * LA + 4 * kq]) = x;
        }
        __syncthreads();
        const int64_t m = m0 + threadIdx.x;
        if (m >= M) continue;
        float l[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) l[c] = bl[c];
        for (int k4 = 0; k4 < CQ; ++k4) {
            const float4 a4 = *reinterpret_cast<const float4*>(&A[threadIdx.x * LA + 4 * k4]);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float* wr = &Ws[(4 * k4 + j) * NC];
#pragma unroll
                for (int c4 = 0; c4 < NC / 4; ++c4) {
                    const float4 w4 = *reinterpret_cast<const float4*>(wr + 4 * c4);
                    l[4 * c4 + 0] = fmaf(av[j], w4.x, l[4 * c4 + 0]);
                    l[4 * c4 + 1] = fmaf(av[j], w4.y, l[4 * c4 + 1]);
                    l[4 * c4 + 2] = fmaf(av[j], w4.z, l[4 * c4 + 2]);
                    l[4 * c4 + 3] = fmaf(av[j], w4.w, l[4 * c4 + 3]);
                }
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < NC; ++c)
            if (c < ncls) mx = fmaxf(mx, l[c]);
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            l[c] = c < ncls ? expf(l[c] - mx) : 0.f;
            s += l[c];
        }
        const float inv = 1.0f / s;
#pragma unroll
        for (int c = 0; c < NC; ++c)
            if (c < ncls) prob[m * ncls + c] = l[c] * inv;
    }
}

// Multi-class head forward on the matrix cores (Cin = 8 KC <= 64, ncls <= 32): one wave per
// 32-pixel subtile, logits^T (32 classes x 32 pixels) = W^T x^T by v_mfma_f32_32x32x2_f32 with
// the kernel as the register-resident A operand and each lane's pixel row as B (lane (lo, hi)
// loads channels 8t + 4hi .. + 3 of pixel lo as float4, t < KC: k step 4t + i is channel
// 8t + 4hi + i on either operand), the bias as the accumulator's start.  Lane (lo, hi) then holds
// 16 of pixel lo's logits (classes acc_row(r, hi)); the softmax combines the two halves with one
// lane swap, and the wave's 32 x ncls probabilities leave through LDS as contiguous float4 runs.
// The next subtile's rows are loaded before this one's products (software prefetch).
// row of accumulator register r of a v_mfma_f32_32x32x2_f32 tile in lane half hi
__device__ __forceinline__ int hx_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }
template <int MODE, int KC>
__global__ __launch_bounds__(256) void head_fwdx_kernel(DView v, int64_t M, int ncls, const float* __restrict__ W,
                                                        const float* __restrict__ bias, float* __restrict__ prob,
                                                        bool vec) {
    __shared__ __attribute__((aligned(16))) float scs[8 * KC], shs[8 * KC];
    __shared__ __attribute__((aligned(16))) float ob[4][32 * 32];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lo = lane & 31, hi = lane >> 5;
    constexpr int CIN = 8 * KC;
    if constexpr (MODE == UNET_VIEW_BNRELU) {
        for (int i = threadIdx.x; i < CIN; i += 256) {
            scs[i] = v.sc0[i];
            shs[i] = v.sh0[i];
        }
    }
    float wa[4 * KC];
#pragma unroll
    for (int t = 0; t < KC; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) wa[4 * t + i] = lo < ncls ? W[(8 * t + 4 * hi + i) * ncls + lo] : 0.f;
    float bl[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int c = hx_row(r, hi);
        bl[r] = (c < ncls && bias) ? bias[c] : 0.f;
    }
    __syncthreads();
    float* o = ob[wave];
    const int64_t nsub = (M + 31) / 32, step = (int64_t)gridDim.x * 4;
    int64_t sub = (int64_t)blockIdx.x * 4 + wave;
    float4 xn[KC];
    auto load = [&](int64_t sb) {
        const int64_t px = sb * 32 + lo;
#pragma unroll
        for (int t = 0; t < KC; ++t) xn[t] = (sb < nsub && px < M) ? ld4(v.src0 + px * CIN + 8 * t + 4 * hi) : f4(0.f);
    };
    load(sub);
    for (; sub < nsub; sub += step) {
        float4 x[KC];
#pragma unroll
        for (int t = 0; t < KC; ++t) x[t] = xn[t];
        load(sub + step);
        if constexpr (MODE == UNET_VIEW_BNRELU) {
#pragma unroll
            for (int t = 0; t < KC; ++t)
                x[t] = bnrelu4(x[t], *reinterpret_cast<const float4*>(&scs[8 * t + 4 * hi]),
                               *reinterpret_cast<const float4*>(&shs[8 * t + 4 * hi]));
        }
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = bl[r];
#pragma unroll
        for (int t = 0; t < KC; ++t) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * t + 0], x[t].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * t + 1], x[t].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * t + 2], x[t].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * t + 3], x[t].w, acc, 0, 0, 0);
        }
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (hx_row(r, hi) < ncls) mx = fmaxf(mx, acc[r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float e[16], sum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            e[r] = hx_row(r, hi) < ncls ? expf(acc[r] - mx) : 0.f;
            sum += e[r];
        }
        sum += __shfl_xor(sum, 32, 64);
        const float inv = 1.0f / sum;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (hx_row(r, hi) < ncls) o[lo * ncls + hx_row(r, hi)] = e[r] * inv;
        __builtin_amdgcn_wave_barrier();
        const int64_t p0 = sub * 32;
        const int cnt = (int)((M - p0 < 32 ? M - p0 : 32) * ncls);
        float* dst = prob + p0 * ncls;
        const int c4n = vec ? cnt >> 2 : 0;
        for (int i = lane; i < c4n; i += 64) st4(dst + 4 * i, *reinterpret_cast<const float4*>(&o[4 * i]));
        for (int i = 4 * c4n + lane; i < cnt; i += 64) dst[i] = o[i];
        __builtin_amdgcn_wave_barrier();
    }
}

// Multi-class head backward over 256-pixel tiles: one thread per pixel forms the softmax-backward
// dlogit (to global for the weight gradient, and into an LDS row of NC + 4 floats), then one
// thread per (pixel, channel quad) forms dx = W dlogit with its 4 x NC kernel values held in
// registers and the pixel's dlogits read 4 at a time (broadcast ds_read_b128).  (The earlier form
// re-read the kernel from LDS for every output and stored dlogit rows 32 floats apart, 32-way
// bank conflicts: 715 us per batch-8 backward, profiles/r4j_cfg4_trace.txt.)
template <int NC, int LOSS>
__global__ __launch_bounds__(256) void head_bwdm_kernel(int64_t M, int64_t hw, int Cin, int ncls,
                                                        const float* __restrict__ W, const float* __restrict__ prob,
                                                        const float* __restrict__ yt, const float* __restrict__ sums,
                                                        float smooth, float gscale, float* __restrict__ dlogit,
                                                        float* __restrict__ dx) {
    constexpr int LD = NC + 4;
    __shared__ __attribute__((aligned(16))) float dls[256 * LD];
    const int CQ = Cin / 4;  // divides 256 (launcher)
    const int kq = threadIdx.x % CQ, pp = threadIdx.x / CQ, PS = 256 / CQ;
    float wr[4][NC];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < NC; ++c) wr[j][c] = c < ncls ? W[(4 * kq + j) * ncls + c] : 0.f;
    for (int64_t m0 = (int64_t)blockIdx.x * 256; m0 < M; m0 += (int64_t)gridDim.x * 256) {
        {
            const int64_t m = m0 + threadIdx.x;
            float p[NC], dl[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                p[c] = 0.f;
                dl[c] = 0.f;
                if (c < ncls && m < M) {
                    p[c] = prob[m * ncls + c];
                    dl[c] = loss_grad<LOSS>(yt[m * ncls + c], sums + ((m / hw) * ncls + c) * 3, smooth, gscale);
                }
            }
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) s = fmaf(dl[c], p[c], s);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                dl[c] = p[c] * (dl[c] - s);
                if (c < ncls && m < M) dlogit[m * ncls + c] = dl[c];
            }
#pragma unroll
            for (int c4 = 0; c4 < NC / 4; ++c4)
                *reinterpret_cast<float4*>(&dls[threadIdx.x * LD + 4 * c4]) =
                    make_float4(dl[4 * c4], dl[4 * c4 + 1], dl[4 * c4 + 2], dl[4 * c4 + 3]);
        }
        __syncthreads();
        for (int p = pp; p < 256; p += PS) {
            const int64_t m = m0 + p;
            if (m >= M) break;
            float4 o = f4(0.f);
#pragma unroll
            for (int c4 = 0; c4 < NC / 4; ++c4) {
                const float4 d = *reinterpret_cast<const float4*>(&dls[p * LD + 4 * c4]);
                const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o.x = fmaf(wr[0][4 * c4 + i], dv[i], o.x);
                    o.y = fmaf(wr[1][4 * c4 + i], dv[i], o.y);
                    o.z = fmaf(wr[2][4 * c4 + i], dv[i], o.z);
                    o.w = fmaf(wr[3][4 * c4 + i], dv[i], o.w);
                }
            }
            st4(dx + m * Cin + 4 * kq, o);
        }
        __syncthreads();
    }
}

// Multi-class head, fully fused backward (ncls <= 24, Cin <= 64 with Cin / 2 dividing 256) over
// 256-pixel tiles -- one pass instead of dlogit out + a weight-gradient GEMM + a column sum (+ the
// BN-backward statistics pass over (dx, z) of the last decoder block):
//   stage  : the tile's prob and y_true rows (ncls contiguous floats a pixel) into LDS, float4;
//   phase 1: one lane per pixel -> dlogit = p (dL/dp - sum_c dL/dp_c p_c), LDS rows of NC + 4;
//   phase 2: one lane per (pixel, channel pair): dx = W dlogit with W's two rows in registers,
//            dW += x dlogit^T in registers across tiles, (STATS) the BN-backward partials of dx;
//            lanes < 8 NC: the tile's dlogit column sums (db), 32 rows each;
//   end    : fixed-order LDS reductions -> per-block partials of dW (Cin x ncls), db (ncls) and
//            (STATS) bnpart[block][0 | 1][c] = sum g | sum g xhat, g = dx [z sc + sh > 0].
typedef float f2v __attribute__((ext_vector_type(2)));
template <int MODE, int NC, int LOSS, bool STATS>
__global__ __launch_bounds__(256) void head_bwdmf_kernel(DView v, int64_t M, int64_t hw, int ncls,
                                                         const float* __restrict__ W, const float* __restrict__ prob,
                                                         const float* __restrict__ yt, const float* __restrict__ sums,
                                                         float smooth, float gscale, bool vec, float* __restrict__ dx,
                                                         float* __restrict__ part_w, float* __restrict__ part_b,
                                                         const float* __restrict__ mu, const float* __restrict__ rs,
                                                         float* __restrict__ bnpart, int ko) {
    main_stream_prio();
    constexpr int LD = NC + 4;
    __shared__ __attribute__((aligned(16))) float Pt[256 * NC];
    __shared__ __attribute__((aligned(16))) float Gt[256 * NC];
    __shared__ __attribute__((aligned(16))) float dls[256 * LD];
    __shared__ float cf[2 * NC * 3];  // the tile's per-(image, class) dice sums (hw >= 256: <= 2 images)
    const bool cfl = hw >= 256;
    const int Cin = v.c0, CP = Cin / 2;
    const int kp = threadIdx.x % CP, pp = threadIdx.x / CP, PS = 256 / CP;
    const int c0 = 2 * kp;
    // the channel pair's kernel rows and weight-gradient sums as float pairs (packed FMAs)
    f2v wr[NC], dw[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        wr[c] = c < ncls ? f2v{W[c0 * ncls + c], W[(c0 + 1) * ncls + c]} : f2v{0.f, 0.f};
        dw[c] = f2v{0.f, 0.f};
    }
    float2 hsc = make_float2(1.f, 1.f), hsh = make_float2(0.f, 0.f), smu = hsh, srs = hsh, s1 = hsh, s2 = hsh;
    if constexpr (MODE == UNET_VIEW_BNRELU) {
        hsc = *reinterpret_cast<const float2*>(v.sc0 + c0);
        hsh = *reinterpret_cast<const float2*>(v.sh0 + c0);
    }
    if constexpr (STATS) {
        if (mu) {
            smu = *reinterpret_cast<const float2*>(mu + c0);
            srs = *reinterpret_cast<const float2*>(rs + c0);
        }
    }
    const int dbc = threadIdx.x % NC, dbq = threadIdx.x / NC;  // db: column, 32-row group
    float dbp = 0.f;
    for (int64_t m0 = (int64_t)blockIdx.x * 256; m0 < M; m0 += (int64_t)gridDim.x * 256) {
        const int np = M - m0 < 256 ? (int)(M - m0) : 256;
        const int cnt = np * ncls;
        const float* pg = prob + m0 * ncls;
        const float* yg = yt + m0 * ncls;
        __syncthreads();
        const int c4n = vec ? cnt >> 2 : 0;
        for (int i0 = threadIdx.x; i0 < c4n; i0 += 256 * 3) {  // 3 + 3 float4 loads in flight
            float4 tp[3], ty[3];
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int i = i0 + 256 * u;
                tp[u] = i < c4n && !(ko & 8) ? ld4(pg + 4 * i) : f4(0.5f);
                ty[u] = i < c4n && !(ko & 8) ? ld4(yg + 4 * i) : f4(0.5f);
            }
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int i = i0 + 256 * u;
                if (i < c4n) {
                    reinterpret_cast<float4*>(Pt)[i] = tp[u];
                    reinterpret_cast<float4*>(Gt)[i] = ty[u];
                }
            }
        }
        for (int i = 4 * c4n + threadIdx.x; i < cnt; i += 256) {
            Pt[i] = pg[i];
            Gt[i] = yg[i];
        }
        const int64_t n0 = m0 / hw;
        if (cfl && threadIdx.x < 2 * ncls * 3) {
            const int64_t o = n0 * ncls * 3 + threadIdx.x;
            cf[threadIdx.x] = o < (M / hw) * ncls * 3 ? sums[o] : 0.f;
        }
        __syncthreads();
        {
            const int p = threadIdx.x;
            float dl[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) dl[c] = 0.f;
            if (p < np && !(ko & 64)) {
                const int64_t nimg = (m0 + p) / hw;
                const float* s3 = cfl ? cf + (nimg - n0) * ncls * 3 : sums + nimg * ncls * 3;
                float s = 0.f;
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    if (c < ncls) {
                        const float g = (ko & 1) ? Gt[p * ncls + c] : loss_grad<LOSS>(Gt[p * ncls + c], s3 + 3 * c, smooth, gscale);
                        dl[c] = g;
                        s = fmaf(g, Pt[p * ncls + c], s);
                    }
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    if (c < ncls) dl[c] = Pt[p * ncls + c] * (dl[c] - s);
            }
#pragma unroll
            for (int c4 = 0; c4 < NC / 4; ++c4)
                *reinterpret_cast<float4*>(&dls[p * LD + 4 * c4]) =
                    make_float4(dl[4 * c4], dl[4 * c4 + 1], dl[4 * c4 + 2], dl[4 * c4 + 3]);
        }
        __syncthreads();
        if (threadIdx.x < 8 * NC && !(ko & 16)) {
            float t = 0.f;
            for (int q = 0; q < 32; ++q) t += dls[(dbq * 32 + q) * LD + dbc];
            dbp += t;
        }
        // input pairs four pixels at a time, the next four loaded before this four's dx stores
        // (vmcnt counts stores too: a load issued after a store waits for it)
        constexpr int U = 4;
        float2 zq[U];
        auto zload = [&](int pb) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                zq[u] = pb + u * PS < np && !(ko & 2)
                            ? *reinterpret_cast<const float2*>(v.src0 + (m0 + pb + u * PS) * Cin + c0)
                            : make_float2(0.5f, 0.5f);
        };
        zload(pp);
        for (int pb = pp; pb < np; pb += U * PS) {
            float2 zc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) zc[u] = zq[u];
            if (pb + U * PS < np) zload(pb + U * PS);
#pragma unroll
            for (int u = 0; u < U; ++u) {
            const int p = pb + u * PS;
            if (p >= np) break;
            const int64_t m = m0 + p;
            const float2 zr = zc[u];
            float2 a = zr;
            if constexpr (MODE == UNET_VIEW_BNRELU)
                a = make_float2(fmaxf(fmaf(zr.x, hsc.x, hsh.x), 0.f), fmaxf(fmaf(zr.y, hsc.y, hsh.y), 0.f));
            f2v o = {0.f, 0.f};
            const f2v a2 = {a.x, a.y};
#pragma unroll
            for (int c4 = 0; c4 < ((ko & 32) ? 0 : NC / 4); ++c4) {
                const float4 d = *reinterpret_cast<const float4*>(&dls[p * LD + 4 * c4]);
                const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const f2v dd = {dv[i], dv[i]};
                    o = __builtin_elementwise_fma(wr[4 * c4 + i], dd, o);
                    dw[4 * c4 + i] = __builtin_elementwise_fma(a2, dd, dw[4 * c4 + i]);
                }
            }
            const float ox = o.x, oy = o.y;
            if (!(ko & 4)) *reinterpret_cast<float2*>(dx + m * Cin + c0) = make_float2(ox, oy);
            if constexpr (STATS) {
                const float gx = a.x > 0.f ? ox : 0.f, gy = a.y > 0.f ? oy : 0.f;
                s1.x += gx;
                s1.y += gy;
                s2.x = fmaf(gx, (zr.x - smu.x) * srs.x, s2.x);
                s2.y = fmaf(gy, (zr.y - smu.y) * srs.y, s2.y);
            }
            }
        }
    }
    // per-block partials, each a fixed-order sum over the block's lanes
    float4* red = reinterpret_cast<float4*>(Pt);  // 256 float4 (Pt holds 256 NC >= 1024 floats)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int c4 = 0; c4 < NC / 4; ++c4) {
            __syncthreads();
            red[threadIdx.x] = j == 0 ? make_float4(dw[4 * c4].x, dw[4 * c4 + 1].x, dw[4 * c4 + 2].x, dw[4 * c4 + 3].x)
                                      : make_float4(dw[4 * c4].y, dw[4 * c4 + 1].y, dw[4 * c4 + 2].y, dw[4 * c4 + 3].y);
            __syncthreads();
            if (threadIdx.x < CP) {
                float4 t = red[threadIdx.x];
                for (int q = threadIdx.x + CP; q < 256; q += CP) t = add4(t, red[q]);
                float* o = part_w + (int64_t)blockIdx.x * Cin * ncls + (2 * threadIdx.x + j) * ncls + 4 * c4;
                if (4 * c4 + 0 < ncls) o[0] = t.x;
                if (4 * c4 + 1 < ncls) o[1] = t.y;
                if (4 * c4 + 2 < ncls) o[2] = t.z;
                if (4 * c4 + 3 < ncls) o[3] = t.w;
            }
        }
    if constexpr (STATS) {
        __syncthreads();
        red[threadIdx.x] = make_float4(s1.x, s1.y, s2.x, s2.y);
        __syncthreads();
        if (threadIdx.x < CP) {
            float4 t = red[threadIdx.x];
            for (int q = threadIdx.x + CP; q < 256; q += CP) t = add4(t, red[q]);
            float* o = bnpart + (int64_t)blockIdx.x * 2 * Cin + 2 * threadIdx.x;
            o[0] = t.x;
            o[1] = t.y;
            o[Cin] = t.z;
            o[Cin + 1] = t.w;
        }
    }
    __syncthreads();
    Gt[threadIdx.x] = dbp;
    __syncthreads();
    if (threadIdx.x < ncls) {
        float t = 0.f;
        for (int q = 0; q < 8; ++q) t += Gt[q * NC + threadIdx.x];
        part_b[(int64_t)blockIdx.x * ncls + threadIdx.x] = t;
    }
}

template <int K>
__device__ __forceinline__ void miou_count(float tv, float q, float thr, unsigned int* h) {
    const long long t = (long long)tv;  // Keras casts to int64 (truncation), then range-checks
    const long long p = thr < 0.f ? (long long)q : (q > thr ? 1 : 0);
    if (t >= 0 && t < K && p >= 0 && p < K) {
        const int b = (int)(t * K + p);
#pragma unroll
        for (int i = 0; i < K * K; ++i) h[i] += b == i ? 1u : 0u;
    }
}
// K x K confusion counts, float4 loads (four elements a lane per load pair; the count % 4 tail by
// the first threads)
template <int K>
__global__ __launch_bounds__(256) void meaniou_small_kernel(const float* __restrict__ yt, const float* __restrict__ yp,
                                                            int64_t count, float thr,
                                                            unsigned long long* __restrict__ conf) {
    unsigned int h[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) h[i] = 0;
    const int64_t n4 = count / 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 t = ld4(yt + 4 * i), q = ld4(yp + 4 * i);
        miou_count<K>(t.x, q.x, thr, h);
        miou_count<K>(t.y, q.y, thr, h);
        miou_count<K>(t.z, q.z, thr, h);
        miou_count<K>(t.w, q.w, thr, h);
    }
    if (blockIdx.x == 0 && threadIdx.x < count - 4 * n4) {
        const int64_t i = 4 * n4 + threadIdx.x;
        miou_count<K>(yt[i], yp[i], thr, h);
    }
    __shared__ unsigned int red[4][K * K];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int b = 0; b < K * K; ++b) {
        unsigned int v = h[b];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) red[wave][b] = v;
    }
    __syncthreads();
    if (threadIdx.x < K * K) {
        const unsigned int s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        if (s) atomicAdd(conf + threadIdx.x, (unsigned long long)s);
    }
}

__global__ __launch_bounds__(256) void meaniou_kernel(const float* __restrict__ yt, const float* __restrict__ yp,
                                                      int64_t count, int K, float thr,
                                                      unsigned long long* __restrict__ conf) {
    __shared__ unsigned int hist[kMaxCls * kMaxCls];
    for (int b = threadIdx.x; b < K * K; b += 256) hist[b] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256) {
        const long long t = (long long)yt[i];
        const float q = yp[i];
        const long long p = thr < 0.f ? (long long)q : (q > thr ? 1 : 0);
        if (t >= 0 && t < K && p >= 0 && p < K) atomicAdd(&hist[t * K + p], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < K * K; b += 256)
        if (hist[b]) atomicAdd(conf + b, (unsigned long long)hist[b]);
}

int grid_for(int64_t work, int cap = 4096) {
    int64_t g = cdiv(work, 256);
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

struct DicePlan {
    int nblk;
    int64_t ppb;
};
DicePlan dice_plan(int n, int64_t hw) {
    DicePlan d;
    int64_t want = cdiv(1024, n);
    int64_t maxb = cdiv(hw, 1024);
    int64_t b = want < maxb ? want : maxb;
    if (b < 1) b = 1;
    d.ppb = cdiv(hw, b);
    d.nblk = (int)cdiv(hw, d.ppb);
    return d;
}

}  // namespace
}  // namespace unet

using namespace unet;

extern "C" int unet_head_fwd(const unet_view* x, int n, int h, int w, int ncls, const float* kernel,
                             const float* bias, float* prob, unet_stream_t stream) {
    if (check_view(x, "unet_head_fwd", true)) return -1;
    UNET_CHECK_ARG(x->mode == UNET_VIEW_PLAIN || x->mode == UNET_VIEW_BNRELU,
                   "unet_head_fwd: input view must be PLAIN or BNRELU");
    UNET_CHECK_ARG(x->drop_rate == 0.f, "unet_head_fwd: dropout on the head input is not supported");
    UNET_CHECK_ARG(x->c0 <= kMaxCin, "unet_head_fwd: Cin %d > %d", x->c0, kMaxCin);
    UNET_CHECK_ARG(ncls >= 1 && ncls <= kMaxCls, "unet_head_fwd: num_classes %d out of [1,%d]", ncls, kMaxCls);
    UNET_CHECK_ARG(kernel && prob && n > 0 && h > 0 && w > 0, "unet_head_fwd: bad args");
    const DView v = make_dview(*x);
    const int64_t M = (int64_t)n * h * w;
    hipStream_t st = as_stream(stream);
    const bool bin_vec = ncls == 1 && (x->c0 == 32 || x->c0 == 64 || x->c0 == 128 || x->c0 == 256) &&
                         ((uintptr_t)x->src0 | (uintptr_t)kernel) % 16 == 0;
    if (bin_vec) {
        const int G = x->c0 / 4;
        const int64_t gb = cdiv(M, (int64_t)16 * (64 / G));
        const int grid = (int)(gb > 4096 ? 4096 : gb);
#define UNET_HB(MODE_)                                                                                       \
    switch (G) {                                                                                             \
        case 8: head_fwd_bin_kernel<MODE_, 8><<<grid, 256, 0, st>>>(v, M, kernel, bias, prob); break;         \
        case 16: head_fwd_bin_kernel<MODE_, 16><<<grid, 256, 0, st>>>(v, M, kernel, bias, prob); break;       \
        case 32: head_fwd_bin_kernel<MODE_, 32><<<grid, 256, 0, st>>>(v, M, kernel, bias, prob); break;       \
        default: head_fwd_bin_kernel<MODE_, 64><<<grid, 256, 0, st>>>(v, M, kernel, bias, prob); break;       \
    }
        if (x->mode == UNET_VIEW_BNRELU) {
            UNET_HB(UNET_VIEW_BNRELU)
        } else {
            UNET_HB(UNET_VIEW_PLAIN)
        }
#undef UNET_HB
        UNET_CHECK_LAUNCH("unet_head_fwd");
        return 0;
    }
    if (ncls > 1 && (x->c0 == 16 || x->c0 == 32 || x->c0 == 64) && ((uintptr_t)x->src0 % 16) == 0) {
        // multi-class on the matrix cores
        const int grid = (int)(cdiv(M, (int64_t)128) > 2048 ? 2048 : cdiv(M, (int64_t)128));
        const bool vec = (uintptr_t)prob % 16 == 0;
#define UNET_HFX(MODE_)                                                                                       \
    switch (x->c0) {                                                                                        \
        case 16: head_fwdx_kernel<MODE_, 2><<<grid, 256, 0, st>>>(v, M, ncls, kernel, bias, prob, vec); break; \
        case 32: head_fwdx_kernel<MODE_, 4><<<grid, 256, 0, st>>>(v, M, ncls, kernel, bias, prob, vec); break; \
        default: head_fwdx_kernel<MODE_, 8><<<grid, 256, 0, st>>>(v, M, ncls, kernel, bias, prob, vec); break; \
    }
        if (x->mode == UNET_VIEW_BNRELU) UNET_HFX(UNET_VIEW_BNRELU)
        else UNET_HFX(UNET_VIEW_PLAIN)
#undef UNET_HFX
        UNET_CHECK_LAUNCH("unet_head_fwd");
        return 0;
    }
    if (ncls > 1 && x->c0 <= 64 && x->c0 % 4 == 0) {  // multi-class: the register-logit kernel
        const int grid = grid_for(M, 4096);
#define UNET_HFM(MODE_, NC_) head_fwdm_kernel<MODE_, NC_><<<grid, 256, 0, st>>>(v, M, ncls, kernel, bias, prob)
#define UNET_HFM_NC(MODE_)                                                                \
    do {                                                                                  \
        if (ncls <= 4) UNET_HFM(MODE_, 4);                                                \
        else if (ncls <= 8) UNET_HFM(MODE_, 8);                                           \
        else if (ncls <= 16) UNET_HFM(MODE_, 16);                                         \
        else if (ncls <= 24) UNET_HFM(MODE_, 24);                                         \
        else UNET_HFM(MODE_, 32);                                                         \
    } while (0)
        if (x->mode == UNET_VIEW_BNRELU) UNET_HFM_NC(UNET_VIEW_BNRELU);
        else UNET_HFM_NC(UNET_VIEW_PLAIN);
#undef UNET_HFM_NC
#undef UNET_HFM
        UNET_CHECK_LAUNCH("unet_head_fwd");
        return 0;
    }
    const int TP = (ncls > 1 ? 4096 : 8192) / x->c0 < 256 ? (ncls > 1 ? 4096 : 8192) / x->c0 : 256;
    int64_t g = cdiv(M, TP);
    const int grid = (int)(g > 4096 ? 4096 : g);
    const bool multi = ncls > 1;
    const size_t smem = ((size_t)kMaxCin * (multi ? kMaxCls : 1) + (multi ? kMaxCls : 1) +
                         (size_t)TP * (x->c0 + 1)) * sizeof(float);
    if (x->mode == UNET_VIEW_BNRELU) {
        if (!multi)
            head_fwd_kernel<UNET_VIEW_BNRELU, 1><<<grid, 256, smem, st>>>(v, M, ncls, kernel, bias, prob);
        else
            head_fwd_kernel<UNET_VIEW_BNRELU, kMaxCls><<<grid, 256, smem, st>>>(v, M, ncls, kernel, bias, prob);
    } else {
        if (!multi)
            head_fwd_kernel<UNET_VIEW_PLAIN, 1><<<grid, 256, smem, st>>>(v, M, ncls, kernel, bias, prob);
        else
            head_fwd_kernel<UNET_VIEW_PLAIN, kMaxCls><<<grid, 256, smem, st>>>(v, M, ncls, kernel, bias, prob);
    }
    UNET_CHECK_LAUNCH("unet_head_fwd");
    return 0;
}

extern "C" size_t unet_dice_workspace(int n, int64_t hw, int ncls) {
    if (n <= 0 || hw <= 0 || ncls <= 0) return 0;
    DicePlan d = dice_plan(n, hw);
    return align_up((size_t)n * d.nblk * 3 * ncls * sizeof(float), 256);
}

extern "C" int unet_dice_fwd(const float* y_true, const float* y_pred, int n, int64_t hw, int ncls, float smooth,
                             float* sums, float* result, void* ws, size_t ws_bytes, unet_stream_t stream) {
    UNET_CHECK_ARG(y_true && y_pred && result && n > 0 && hw > 0, "unet_dice_fwd: bad args");
    UNET_CHECK_ARG(ncls >= 1 && ncls <= kMaxCls, "unet_dice_fwd: num_classes %d out of [1,%d]", ncls, kMaxCls);
    const size_t need = unet_dice_workspace(n, hw, ncls);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_dice_fwd: workspace %zu < %zu", ws_bytes, need);
    DicePlan d = dice_plan(n, hw);
    hipStream_t st = as_stream(stream);
    float* part = static_cast<float*>(ws);
    dim3 grid(d.nblk, n);
    if (ncls == 1)
        dice_partial_kernel<1><<<grid, 256, 0, st>>>(y_true, y_pred, hw, ncls, d.ppb, part);
    else if (ncls <= 4)
        dice_partial_m_kernel<4><<<grid, 256, 0, st>>>(y_true, y_pred, hw, ncls, d.ppb, part);
    else if (ncls <= 8)
        dice_partial_m_kernel<8><<<grid, 256, 0, st>>>(y_true, y_pred, hw, ncls, d.ppb, part);
    else if (ncls <= 16)
        dice_partial_m_kernel<16><<<grid, 256, 0, st>>>(y_true, y_pred, hw, ncls, d.ppb, part);
    else if (ncls <= 24)
        dice_partial_m_kernel<24><<<grid, 256, 0, st>>>(y_true, y_pred, hw, ncls, d.ppb, part);
    else
        dice_partial_m_kernel<32><<<grid, 256, 0, st>>>(y_true, y_pred, hw, ncls, d.ppb, part);
    UNET_CHECK_LAUNCH("unet_dice_fwd(partial)");
    dice_finalize_kernel<<<1, n * ncls >= 64 ? 1024 : 256, 0, st>>>(part, n, d.nblk, ncls, smooth, sums, result);
    UNET_CHECK_LAUNCH("unet_dice_fwd(finalize)");
    return 0;
}

extern "C" size_t unet_head_bwd_workspace(int n, int h, int w, int cin, int ncls) {
    if (n <= 0 || h <= 0 || w <= 0 || cin <= 0 || ncls <= 0) return 0;
    const int64_t M = (int64_t)n * h * w;
    const size_t dl = align_up((size_t)M * ncls * sizeof(float), 256);
    size_t a = head_wgrad_workspace(M, cin, ncls);
    size_t b = colsum_workspace(M, ncls);
    const size_t fused = (align_up((size_t)1024 * cin * ncls, 64) + align_up((size_t)1024 * ncls, 64)) * sizeof(float);
    const size_t gen = dl + (a > b ? a : b);
    return align_up(fused > gen ? fused : gen, 256);
}

namespace {
int head_bwd_grid(int64_t M) {
    const int64_t g = cdiv(M, 256);
    return (int)(g > 1024 ? 1024 : g);
}
// the fused multi-class backward (head_bwdmf_kernel) covers this head
bool head_bwdmf_ok(const unet_view* x, int ncls) {
    return ncls > 1 && ncls <= 24 && x->c0 <= 64 && x->c0 % 4 == 0 && 256 % (x->c0 / 2) == 0;
}
int head_bwdmf_grid(int64_t M) {  // 2 blocks a CU (77 KB of LDS at 24 classes): one wave of blocks
    const int64_t g = cdiv(M, 256);
    return (int)(g > 512 ? 512 : g);
}
int head_bwd_impl(const unet_view* x, int n, int h, int w, int ncls, const float* kernel, const float* prob,
                  const float* y_true, const float* sums, float smooth, int loss_kind, float loss_scale, float* dx,
                  float* dkernel, float* dbias, void* ws, size_t ws_bytes, const float* mu, const float* rs,
                  float* bnpart, unet_stream_t stream, float* dlogit = nullptr);
}  // namespace

extern "C" int unet_head_bwd_bnstats_slabs(const unet_view* x, int n, int h, int w, int ncls) {
    if (!x || x->mode != UNET_VIEW_BNRELU || n <= 0 || h <= 0 || w <= 0) return 0;
    if (ncls > 1) return head_bwdmf_ok(x, ncls) ? head_bwdmf_grid((int64_t)n * h * w) : 0;
    if (ncls != 1 || x->c0 % 4 || x->c0 > kMaxCin || 256 % (x->c0 / 4)) return 0;
    return head_bwd_grid((int64_t)n * h * w);
}

extern "C" int unet_head_bwd_bnstats(const unet_view* x, int n, int h, int w, int ncls, const float* kernel,
                                     const float* prob, const float* y_true, const float* sums, float smooth,
                                     int loss_kind, float loss_scale, float* dx, float* dlogit, float* dkernel,
                                     float* dbias, const float* mean,
                                     const float* rstd, float* bn_partials, void* ws, size_t ws_bytes,
                                     unet_stream_t stream) {
    UNET_CHECK_ARG(unet_head_bwd_bnstats_slabs(x, n, h, w, ncls) > 0,
                   "unet_head_bwd_bnstats: needs a BNRELU view with Cin %% 4 == 0 (multi-class: <= 24 classes, "
                   "Cin in {4, 8, 16, 32, 64})");
    UNET_CHECK_ARG(ncls == 1 || dlogit == nullptr, "unet_head_bwd_bnstats: the dlogit form is binary-only");
    UNET_CHECK_ARG(bn_partials, "unet_head_bwd_bnstats: null bn_partials");
    UNET_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "unet_head_bwd_bnstats: mean and rstd go together");
    UNET_CHECK_ARG((dx == nullptr) != (dlogit == nullptr), "unet_head_bwd_bnstats: give exactly one of dx, dlogit");
    return head_bwd_impl(x, n, h, w, ncls, kernel, prob, y_true, sums, smooth, loss_kind, loss_scale, dx, dkernel,
                         dbias, ws, ws_bytes, mean, rstd, bn_partials, stream, dlogit);
}

extern "C" int unet_head_bwd(const unet_view* x, int n, int h, int w, int ncls, const float* kernel,
                             const float* prob, const float* y_true, const float* sums, float smooth, int loss_kind,
                             float loss_scale, float* dx, float* dkernel, float* dbias, void* ws, size_t ws_bytes,
                             unet_stream_t stream) {
    return head_bwd_impl(x, n, h, w, ncls, kernel, prob, y_true, sums, smooth, loss_kind, loss_scale, dx, dkernel,
                         dbias, ws, ws_bytes, nullptr, nullptr, nullptr, stream);
}

namespace {
int head_bwd_impl(const unet_view* x, int n, int h, int w, int ncls, const float* kernel, const float* prob,
                  const float* y_true, const float* sums, float smooth, int loss_kind, float loss_scale, float* dx,
                  float* dkernel, float* dbias, void* ws, size_t ws_bytes, const float* mu, const float* rs,
                  float* bnpart, unet_stream_t stream, float* dlogit) {
    if (check_view(x, "unet_head_bwd", true)) return -1;
    if (dlogit) dx = dlogit;  // (unet_head_bwd_bnstats' rank-one form: the STATS kernel writes dlogit)
    UNET_CHECK_ARG(loss_scale > 0.0f && loss_scale < 1e30f, "unet_head_bwd: loss_scale must be finite and > 0");
    UNET_CHECK_ARG(x->mode == UNET_VIEW_PLAIN || x->mode == UNET_VIEW_BNRELU,
                   "unet_head_bwd: input view must be PLAIN or BNRELU");
    UNET_CHECK_ARG(x->c0 <= kMaxCin, "unet_head_bwd: Cin %d > %d", x->c0, kMaxCin);
    UNET_CHECK_ARG(ncls >= 1 && ncls <= kMaxCls, "unet_head_bwd: num_classes out of range");
    UNET_CHECK_ARG(loss_kind == UNET_LOSS_DICE || loss_kind == UNET_LOSS_IOU, "unet_head_bwd: bad loss_kind");
    UNET_CHECK_ARG(kernel && prob && y_true && sums && dx && dkernel && dbias, "unet_head_bwd: null pointer");
    const size_t need = unet_head_bwd_workspace(n, h, w, x->c0, ncls);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_head_bwd: workspace %zu < %zu", ws_bytes, need);
    const int64_t M = (int64_t)n * h * w;
    const int64_t hw = (int64_t)h * w;
    hipStream_t st = as_stream(stream);
    // d(mean over the n*ncls (image, class) terms)/dp, times the caller's loss scale (data
    // parallelism with unequal shards: n_local * world / n_global, 1 otherwise)
    const float gscale = loss_scale / (float)((int64_t)n * ncls);
    const DView v = make_dview(*x);
    const int CQ = x->c0 / 4;
    if (ncls == 1 && 256 % CQ == 0) {
        const int grid = head_bwd_grid(M);
        float* part_w = static_cast<float*>(ws);
        float* part_b = part_w + align_up((size_t)grid * x->c0, 64);
#define UNET_HB1(MODE, L)                                                                                     \
    head_bwd1_kernel<MODE, L><<<grid, 256, 0, st>>>(v, M, hw, kernel, prob, y_true, sums, smooth, gscale, dx, \
                                                     part_w, part_b)
#define UNET_HB1S(L)                                                                                          \
    head_bwd1_kernel<UNET_VIEW_BNRELU, L, true><<<grid, 256, 0, st>>>(v, M, hw, kernel, prob, y_true, sums,   \
                                                                      smooth, gscale, dx, part_w, part_b, mu, rs, bnpart)
#define UNET_HB1D(L)                                                                                          \
    head_bwd1_kernel<UNET_VIEW_BNRELU, L, true, true><<<grid, 256, 0, st>>>(v, M, hw, kernel, prob, y_true,   \
                                                                            sums, smooth, gscale, dlogit, part_w, \
                                                                            part_b, mu, rs, bnpart)
        if (bnpart && dlogit) {
            if (loss_kind == UNET_LOSS_DICE) UNET_HB1D(UNET_LOSS_DICE);
            else UNET_HB1D(UNET_LOSS_IOU);
        } else if (bnpart) {
            if (loss_kind == UNET_LOSS_DICE) UNET_HB1S(UNET_LOSS_DICE);
            else UNET_HB1S(UNET_LOSS_IOU);
        } else if (x->mode == UNET_VIEW_BNRELU) {
            if (loss_kind == UNET_LOSS_DICE) UNET_HB1(UNET_VIEW_BNRELU, UNET_LOSS_DICE);
            else UNET_HB1(UNET_VIEW_BNRELU, UNET_LOSS_IOU);
        } else {
            if (loss_kind == UNET_LOSS_DICE) UNET_HB1(UNET_VIEW_PLAIN, UNET_LOSS_DICE);
            else UNET_HB1(UNET_VIEW_PLAIN, UNET_LOSS_IOU);
        }
#undef UNET_HB1
#undef UNET_HB1S
#undef UNET_HB1D
        UNET_CHECK_LAUNCH("unet_head_bwd");
        return reduce_slabs_pair(part_w, x->c0, dkernel, part_b, 1, dbias, grid, st);
    }
    if (head_bwdmf_ok(x, ncls)) {
        const int grid = head_bwdmf_grid(M);
        float* part_w = static_cast<float*>(ws);
        float* part_b = part_w + align_up((size_t)grid * x->c0 * ncls, 64);
        const bool vec = ((uintptr_t)prob | (uintptr_t)y_true) % 16 == 0;
        const int ko = lab_knob("UNET_HEAD_KO", 0);  // lab timing knock-outs (0 in the product)
#define UNET_HMF(MODE_, NC_, L_, S_)                                                                            \
    head_bwdmf_kernel<MODE_, NC_, L_, S_><<<grid, 256, 0, st>>>(v, M, hw, ncls, kernel, prob, y_true, sums, smooth, \
                                                              gscale, vec, dx, part_w, part_b, mu, rs, bnpart, ko)
#define UNET_HMF_NC(MODE_, L_, S_)                   \
    do {                                             \
        if (ncls <= 4) UNET_HMF(MODE_, 4, L_, S_);   \
        else if (ncls <= 8) UNET_HMF(MODE_, 8, L_, S_);  \
        else if (ncls <= 16) UNET_HMF(MODE_, 16, L_, S_); \
        else UNET_HMF(MODE_, 24, L_, S_);            \
    } while (0)
#define UNET_HMF_L(MODE_, S_)                                            \
    do {                                                                 \
        if (loss_kind == UNET_LOSS_DICE) UNET_HMF_NC(MODE_, UNET_LOSS_DICE, S_); \
        else UNET_HMF_NC(MODE_, UNET_LOSS_IOU, S_);                     \
    } while (0)
        if (bnpart) UNET_HMF_L(UNET_VIEW_BNRELU, true);
        else if (x->mode == UNET_VIEW_BNRELU) UNET_HMF_L(UNET_VIEW_BNRELU, false);
        else UNET_HMF_L(UNET_VIEW_PLAIN, false);
#undef UNET_HMF_L
#undef UNET_HMF_NC
#undef UNET_HMF
        UNET_CHECK_LAUNCH("unet_head_bwd");
        const int64_t L = (int64_t)x->c0 * ncls;
        return reduce_slabs_pair(part_w, L, dkernel, part_b, ncls, dbias, grid, st);
    }
    float* dlg = static_cast<float*>(ws);
    const size_t dl = align_up((size_t)M * ncls * sizeof(float), 256);
    void* ws2 = static_cast<char*>(ws) + dl;
    const size_t ws2_bytes = ws_bytes - dl;
    int64_t g = cdiv(M, 256);
    const int grid = (int)(g > 4096 ? 4096 : g);
#define UNET_HB(NC, L)                                                                                        \
    head_bwd_kernel<NC, L><<<grid, 256, 0, st>>>(M, hw, x->c0, ncls, kernel, prob, y_true, sums, smooth, gscale, \
                                                 dlg, dx)
    if (ncls > 1 && 256 % CQ == 0) {  // multi-class: kernel in registers, dlogit rows in LDS
        const int gridm = (int)(cdiv(M, 256) > 2048 ? 2048 : cdiv(M, 256));
#define UNET_HBM(NC_, L_)                                                                                     \
    head_bwdm_kernel<NC_, L_><<<gridm, 256, 0, st>>>(M, hw, x->c0, ncls, kernel, prob, y_true, sums, smooth, \
                                                     gscale, dlg, dx)
#define UNET_HBM_NC(L_)                                        \
    do {                                                       \
        if (ncls <= 4) UNET_HBM(4, L_);                        \
        else if (ncls <= 8) UNET_HBM(8, L_);                   \
        else if (ncls <= 16) UNET_HBM(16, L_);                 \
        else if (ncls <= 24) UNET_HBM(24, L_);                 \
        else UNET_HBM(32, L_);                                 \
    } while (0)
        if (loss_kind == UNET_LOSS_DICE) UNET_HBM_NC(UNET_LOSS_DICE);
        else UNET_HBM_NC(UNET_LOSS_IOU);
#undef UNET_HBM_NC
#undef UNET_HBM
    } else if (ncls == 1) {
        if (loss_kind == UNET_LOSS_DICE) UNET_HB(1, UNET_LOSS_DICE);
        else UNET_HB(1, UNET_LOSS_IOU);
    } else {
        if (loss_kind == UNET_LOSS_DICE) UNET_HB(kMaxCls, UNET_LOSS_DICE);
        else UNET_HB(kMaxCls, UNET_LOSS_IOU);
    }
#undef UNET_HB
    UNET_CHECK_LAUNCH("unet_head_bwd");
    int rc = head_wgrad(x, M, dlg, ncls, dkernel, ws2, ws2_bytes, st);
    if (rc) return rc;
    return colsum(dlg, M, ncls, dbias, ws2, ws2_bytes, st);
}
}  // namespace

extern "C" int unet_meaniou_update(const float* y_true, const float* y_pred, int64_t count, int num_classes,
                                   float threshold, uint64_t* confusion, unet_stream_t stream) {
    UNET_CHECK_ARG(y_true && y_pred && confusion && count >= 0, "unet_meaniou_update: bad args");
    UNET_CHECK_ARG(num_classes >= 1 && num_classes <= kMaxCls, "unet_meaniou_update: num_classes out of [1,%d]",
                   kMaxCls);
    if (count == 0) return 0;
    hipStream_t st = as_stream(stream);
    const int grid = grid_for(count, 2048);
    auto* conf = reinterpret_cast<unsigned long long*>(confusion);
    if (num_classes == 2 && ((uintptr_t)y_true | (uintptr_t)y_pred) % 16 == 0)
        meaniou_small_kernel<2><<<grid_for(cdiv(count, 4), 2048), 256, 0, st>>>(y_true, y_pred, count, threshold, conf);
    else
        meaniou_kernel<<<grid, 256, 0, st>>>(y_true, y_pred, count, num_classes, threshold, conf);
    UNET_CHECK_LAUNCH("unet_meaniou_update");
    return 0;
}
