// Depthwise 3x3 half of SeparableConv2D (reference: model/u_net.py:14-20; Keras
// SeparableConv2D = tf.nn.separable_conv2d, depthwise stage = DepthwiseConv2dNative,
// stride 1, 'same' zero padding, depth_multiplier 1, kernel (3,3,C,1)).
//
// HBM-bound (18 flop per output element): each lane owns one (pixel, 4-channel)
// quad; consecutive lanes walk consecutive channel quads of one pixel, so every
// wave reads/writes contiguous NHWC rows (coalesced 16-B accesses).  The 3x3 halo
// re-reads hit L1/L2.  The input is read through an activation view (BN+ReLU,
// max-pool, concat, dropout fused on load).
#include "view.h"

namespace unet {

namespace {

constexpr int kThreads = 256;

// 32-bit index math (the launchers check that every tensor has < 2^31 elements)
__device__ __forceinline__ void decompose(int p, int H, int W, int& n, int& h, int& w) {
    w = p % W;
    const int t = p / W;
    h = t % H;
    n = t / H;
}

template <int MODE, bool DROP>
__device__ __forceinline__ float4 tap4(const DView& v, int n, int hh, int ww, int H, int W, int c) {
    float4 x = view_load4<MODE>(v, n, hh, ww, H, W, c);
    if constexpr (DROP) {
        const uint64_t i = ((uint64_t)((int64_t)(n * H + hh) * W + ww)) * v.C + c;
        x = mul4(x, drop_mult4(v.seed, i, v.rate, v.inv_keep));
    }
    return x;
}
template <int MODE, bool DROP>
__device__ __forceinline__ float tap1(const DView& v, int n, int hh, int ww, int H, int W, int c) {
    float x = view_load1<MODE>(v, n, hh, ww, H, W, c);
    if constexpr (DROP)
        x *= drop_mult(v.seed, ((uint64_t)((int64_t)(n * H + hh) * W + ww)) * v.C + c, v.rate, v.inv_keep);
    return x;
}

// ------------------------------------------------------------------ forward ----
template <int MODE, bool DROP, bool VEC>
__global__ __launch_bounds__(kThreads) void dw_fwd_kernel(DView v, int N, int H, int W,
                                                          const float* __restrict__ K,
                                                          float* __restrict__ Y) {
    const int C = v.C;
    const int CQ = VEC ? C / 4 : C;
    const int total = N * H * W * CQ;
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < total; idx += gridDim.x * kThreads) {
        const int cq = idx % CQ;
        const int p = idx / CQ;
        int n, h, w;
        decompose(p, H, W, n, h, w);
        if constexpr (VEC) {
            const int c = cq * 4;
            float4 acc = f4(0.f);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int hh = h + i - 1;
                if (hh < 0 || hh >= H) continue;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int ww = w + j - 1;
                    if (ww < 0 || ww >= W) continue;
                    acc = fma4(tap4<MODE, DROP>(v, n, hh, ww, H, W, c), ld4(K + (i * 3 + j) * C + c), acc);
                }
            }
            st4(Y + p * C + c, acc);
        } else {
            const int c = cq;
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int hh = h + i - 1;
                if (hh < 0 || hh >= H) continue;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int ww = w + j - 1;
                    if (ww < 0 || ww >= W) continue;
                    acc = fmaf(tap1<MODE, DROP>(v, n, hh, ww, H, W, c), K[(i * 3 + j) * C + c], acc);
                }
            }
            Y[p * C + c] = acc;
        }
    }
}

// ------------------------------------------------------------ backward data ----
// dx[h,w] = sum_{i,j} dy[h-i+1, w-j+1] * k[i,j]; then dropout, then routed per view.
template <int MODE, bool DROP, bool VEC>
__global__ __launch_bounds__(kThreads) void dw_bwd_data_kernel(DView v, int N, int H, int W,
                                                               const float* __restrict__ K,
                                                               const float* __restrict__ dY,
                                                               float* __restrict__ dx0,
                                                               float* __restrict__ dx1) {
    const int C = v.C;
    const int CQ = VEC ? C / 4 : C;
    const int total = N * H * W * CQ;
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < total; idx += gridDim.x * kThreads) {
        const int cq = idx % CQ;
        const int p = idx / CQ;
        int n, h, w;
        decompose(p, H, W, n, h, w);
        if constexpr (VEC) {
            const int c = cq * 4;
            float4 acc = f4(0.f);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int hh = h - i + 1;
                if (hh < 0 || hh >= H) continue;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int ww = w - j + 1;
                    if (ww < 0 || ww >= W) continue;
                    acc = fma4(ld4(dY + ((int64_t)(n * H + hh) * W + ww) * C + c), ld4(K + (i * 3 + j) * C + c),
                               acc);
                }
            }
            if constexpr (DROP) {
                const uint64_t li = (uint64_t)p * C + c;
                acc = mul4(acc, drop_mult4(v.seed, li, v.rate, v.inv_keep));
            }
            if constexpr (MODE == UNET_VIEW_PLAIN || MODE == UNET_VIEW_BNRELU) {
                st4(dx0 + p * C + c, acc);
            } else if constexpr (MODE == UNET_VIEW_CONCAT) {
                if (c < v.c0)
                    st4(dx0 + p * v.c0 + c, acc);
                else
                    st4(dx1 + p * v.c1 + (c - v.c0), acc);
            } else {  // POOL_BNRELU: route to the first max of the 2x2 window (row-major scan)
                const int W2 = 2 * W;
                const int64_t b = ((int64_t)(n * 2 * H + 2 * h) * W2 + 2 * w) * v.c0 + c;
                const int64_t off[4] = {0, v.c0, (int64_t)W2 * v.c0, (int64_t)W2 * v.c0 + v.c0};
                const float4 sc = ld4(v.sc0 + c), sh = ld4(v.sh0 + c);
                float4 xv[4], g[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    xv[q] = bnrelu4(ld4(v.src0 + b + off[q]), sc, sh);
                    g[q] = ld4(dx0 + b + off[q]);
                }
                float best;
                int arg;
#define UNET_POOL_ROUTE(comp)                                        \
    best = xv[0].comp;                                               \
    arg = 0;                                                         \
    if (xv[1].comp > best) { best = xv[1].comp; arg = 1; }           \
    if (xv[2].comp > best) { best = xv[2].comp; arg = 2; }           \
    if (xv[3].comp > best) { best = xv[3].comp; arg = 3; }           \
    g[0].comp += arg == 0 ? acc.comp : 0.f;                          \
    g[1].comp += arg == 1 ? acc.comp : 0.f;                          \
    g[2].comp += arg == 2 ? acc.comp : 0.f;                          \
    g[3].comp += arg == 3 ? acc.comp : 0.f;
                UNET_POOL_ROUTE(x)
                UNET_POOL_ROUTE(y)
                UNET_POOL_ROUTE(z)
                UNET_POOL_ROUTE(w)
#undef UNET_POOL_ROUTE
#pragma unroll
                for (int q = 0; q < 4; ++q) st4(dx0 + b + off[q], g[q]);
            }
        } else {
            const int c = cq;
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int hh = h - i + 1;
                if (hh < 0 || hh >= H) continue;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int ww = w - j + 1;
                    if (ww < 0 || ww >= W) continue;
                    acc = fmaf(dY[((int64_t)(n * H + hh) * W + ww) * C + c], K[(i * 3 + j) * C + c], acc);
                }
            }
            if constexpr (DROP) acc *= drop_mult(v.seed, (uint64_t)p * C + c, v.rate, v.inv_keep);
            if constexpr (MODE == UNET_VIEW_PLAIN || MODE == UNET_VIEW_BNRELU) {
                dx0[p * C + c] = acc;
            } else if constexpr (MODE == UNET_VIEW_CONCAT) {
                if (c < v.c0)
                    dx0[p * v.c0 + c] = acc;
                else
                    dx1[p * v.c1 + (c - v.c0)] = acc;
            } else {
                const int W2 = 2 * W;
                const int64_t b = ((int64_t)(n * 2 * H + 2 * h) * W2 + 2 * w) * v.c0 + c;
                const int64_t off[4] = {0, v.c0, (int64_t)W2 * v.c0, (int64_t)W2 * v.c0 + v.c0};
                const float sc = v.sc0[c], sh = v.sh0[c];
                float best = bnrelu(v.src0[b], sc, sh);
                int arg = 0;
#pragma unroll
                for (int q = 1; q < 4; ++q) {
                    float xq = bnrelu(v.src0[b + off[q]], sc, sh);
                    if (xq > best) { best = xq; arg = q; }
                }
                dx0[b + off[arg]] += acc;
            }
        }
    }
}

// ---------------------------------------------------------- backward filter ----
// dk[i,j,c] = sum_p x(p + (i-1, j-1))[c] * dy[p][c].  Block = CT channel lanes x PL
// pixel lanes over a pixel chunk; fixed-order LDS reduction -> partial[chunk][9][C].
template <int MODE, bool DROP, bool VEC>
__global__ __launch_bounds__(kThreads) void dw_bwd_filter_kernel(DView v, int N, int H, int W,
                                                                 const float* __restrict__ dY,
                                                                 float* __restrict__ part, int64_t ppc) {
    const int C = v.C;
    const int CQ = VEC ? C / 4 : C;
    const int CT = CQ < 64 ? CQ : 64;
    const int PL = kThreads / CT;
    const int tid = threadIdx.x;
    const int cl = tid % CT;
    const int pl = tid / CT;
    const int cq = blockIdx.x * CT + cl;
    const int P = N * H * W;
    const int p0 = blockIdx.y * (int)ppc;
    const int p1 = p0 + (int)ppc < P ? p0 + (int)ppc : P;
    __shared__ float4 red[kThreads];

    const bool active = pl < PL && cq < CQ;
    float4 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f4(0.f);
    if (active) {
        for (int p = p0 + pl; p < p1; p += PL) {
            int n, h, w;
            decompose(p, H, W, n, h, w);
            if constexpr (VEC) {
                const int c = cq * 4;
                const float4 g = ld4(dY + p * C + c);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int hh = h + i - 1;
                    if (hh < 0 || hh >= H) continue;
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const int ww = w + j - 1;
                        if (ww < 0 || ww >= W) continue;
                        acc[i * 3 + j] = fma4(tap4<MODE, DROP>(v, n, hh, ww, H, W, c), g, acc[i * 3 + j]);
                    }
                }
            } else {
                const int c = cq;
                const float g = dY[p * C + c];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int hh = h + i - 1;
                    if (hh < 0 || hh >= H) continue;
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const int ww = w + j - 1;
                        if (ww < 0 || ww >= W) continue;
                        acc[i * 3 + j].x = fmaf(tap1<MODE, DROP>(v, n, hh, ww, H, W, c), g, acc[i * 3 + j].x);
                    }
                }
            }
        }
    }
    // fixed-order reduction over the PL pixel lanes, one tap at a time
    float* out = part + (int64_t)blockIdx.y * 9 * C;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        red[tid] = acc[t];
        __syncthreads();
        if (pl == 0 && cq < CQ) {
            float4 s = red[cl];
            for (int q = 1; q < PL; ++q) s = add4(s, red[q * CT + cl]);
            if constexpr (VEC)
                st4(out + t * C + cq * 4, s);
            else
                out[t * C + cq] = s.x;
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------- materialize ----
template <int MODE, bool DROP, bool VEC>
__global__ __launch_bounds__(kThreads) void view_materialize_kernel(DView v, int N, int H, int W,
                                                                    float* __restrict__ out) {
    const int C = v.C;
    const int CQ = VEC ? C / 4 : C;
    const int total = N * H * W * CQ;
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < total; idx += gridDim.x * kThreads) {
        const int cq = idx % CQ;
        const int p = idx / CQ;
        int n, h, w;
        decompose(p, H, W, n, h, w);
        if constexpr (VEC)
            st4(out + p * C + cq * 4, tap4<MODE, DROP>(v, n, h, w, H, W, cq * 4));
        else
            out[p * C + cq] = tap1<MODE, DROP>(v, n, h, w, H, W, cq);
    }
}

struct FilterPlan {
    int ctiles;
    int64_t chunks, ppc;
};
FilterPlan filter_plan(int n, int h, int w, int c) {
    const bool vec = c % 4 == 0;
    const int CQ = vec ? c / 4 : c;
    const int CT = CQ < 64 ? CQ : 64;
    FilterPlan fp;
    fp.ctiles = (int)cdiv(CQ, CT);
    const int64_t P = (int64_t)n * h * w;
    int64_t want = cdiv(2048, fp.ctiles);
    int64_t maxc = cdiv(P, 256);  // at least ~256 pixels per chunk
    fp.chunks = want < maxc ? want : maxc;
    if (fp.chunks < 1) fp.chunks = 1;
    fp.ppc = cdiv(P, fp.chunks);
    fp.chunks = cdiv(P, fp.ppc);
    return fp;
}

int grid_for(int64_t work) {
    int64_t g = cdiv(work, kThreads);
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

// ------------------------------------------------------------ dispatch ----
#define UNET_DW_DISPATCH(KERNEL, GRID, ...)                                                        \
    do {                                                                                           \
        const bool drop_ = x->drop_rate > 0.f;                                                     \
        switch (x->mode) {                                                                         \
            case UNET_VIEW_PLAIN:                                                                  \
                if (drop_) {                                                                       \
                    if (vec) KERNEL<UNET_VIEW_PLAIN, true, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);  \
                    else KERNEL<UNET_VIEW_PLAIN, true, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);     \
                } else {                                                                           \
                    if (vec) KERNEL<UNET_VIEW_PLAIN, false, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__); \
                    else KERNEL<UNET_VIEW_PLAIN, false, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);    \
                }                                                                                  \
                break;                                                                             \
            case UNET_VIEW_BNRELU:                                                                 \
                if (drop_) {                                                                       \
                    if (vec) KERNEL<UNET_VIEW_BNRELU, true, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);  \
                    else KERNEL<UNET_VIEW_BNRELU, true, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);     \
                } else {                                                                           \
                    if (vec) KERNEL<UNET_VIEW_BNRELU, false, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__); \
                    else KERNEL<UNET_VIEW_BNRELU, false, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);    \
                }                                                                                  \
                break;                                                                             \
            case UNET_VIEW_POOL_BNRELU:                                                            \
                if (drop_) {                                                                       \
                    if (vec) KERNEL<UNET_VIEW_POOL_BNRELU, true, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);  \
                    else KERNEL<UNET_VIEW_POOL_BNRELU, true, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);     \
                } else {                                                                           \
                    if (vec) KERNEL<UNET_VIEW_POOL_BNRELU, false, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__); \
                    else KERNEL<UNET_VIEW_POOL_BNRELU, false, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);    \
                }                                                                                  \
                break;                                                                             \
            default:                                                                               \
                if (drop_) {                                                                       \
                    if (vec) KERNEL<UNET_VIEW_CONCAT, true, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);  \
                    else KERNEL<UNET_VIEW_CONCAT, true, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);     \
                } else {                                                                           \
                    if (vec) KERNEL<UNET_VIEW_CONCAT, false, true><<<GRID, kThreads, 0, st>>>(__VA_ARGS__); \
                    else KERNEL<UNET_VIEW_CONCAT, false, false><<<GRID, kThreads, 0, st>>>(__VA_ARGS__);    \
                }                                                                                  \
                break;                                                                             \
        }                                                                                          \
    } while (0)

static bool view_vec(const unet_view* x) {
    if (x->mode == UNET_VIEW_CONCAT) return x->c0 % 4 == 0 && x->c1 % 4 == 0;
    return x->c0 % 4 == 0;
}

int dw_tiled_fwd(const DView& v, int mode, bool drop, int N, int H, int W, const float* K, float* Y, hipStream_t st);
int dw_tiled_bwd_data(const DView& v, int mode, bool drop, int N, int H, int W, const float* K, const float* dY,
                      float* dx0, float* dx1, hipStream_t st);
size_t dw_tiled_filter_partials(int N, int H, int W, int C);
int dw_tiled_bwd_filter(const DView& v, int mode, bool drop, int N, int H, int W, const float* dY, float* part,
                        int* S_out, hipStream_t st);
bool dw_tiled_ok(int C);
int dw_tiled_bwd_data_bnstats(const DView& v, int mode, bool drop, int N, int H, int W, const float* K,
                              const float* dY, float* dx0, const float* mu, const float* rs, float* bnpart,
                              hipStream_t st, float* dwpart = nullptr);
size_t dw_tiled_ntiles(int N, int H, int W, int C);

static int check_dims(const unet_view* x, int n, int h, int w, const char* op) {
    UNET_CHECK_ARG(n > 0 && h > 0 && w > 0, "%s: bad shape n=%d h=%d w=%d", op, n, h, w);
    const int64_t C = x->c0 + (x->mode == UNET_VIEW_CONCAT ? x->c1 : 0);
    const int64_t src = (int64_t)n * h * w * C * (x->mode == UNET_VIEW_POOL_BNRELU ? 4 : 1);
    UNET_CHECK_ARG(src < (int64_t(1) << 31), "%s: tensor too large for 32-bit indexing", op);
    return 0;
}

}  // namespace unet

using namespace unet;

extern "C" int unet_dwconv3x3_fwd(const unet_view* x, int n, int h, int w, const float* dw_kernel, float* y,
                                  unet_stream_t stream) {
    if (check_view(x, "unet_dwconv3x3_fwd") || check_dims(x, n, h, w, "unet_dwconv3x3_fwd")) return -1;
    UNET_CHECK_ARG(dw_kernel && y, "unet_dwconv3x3_fwd: null kernel/output");
    const DView v = make_dview(*x);
    const bool vec = view_vec(x);
    if (vec && dw_tiled_ok(v.C))
        return dw_tiled_fwd(v, x->mode, x->drop_rate > 0.f, n, h, w, dw_kernel, y, as_stream(stream));
    const int64_t work = (int64_t)n * h * w * (vec ? v.C / 4 : v.C);
    hipStream_t st = as_stream(stream);
    const int grid = grid_for(work);
    UNET_DW_DISPATCH(dw_fwd_kernel, grid, v, n, h, w, dw_kernel, y);
    UNET_CHECK_LAUNCH("unet_dwconv3x3_fwd");
    return 0;
}

extern "C" int unet_view_materialize(const unet_view* x, int n, int h, int w, float* out, unet_stream_t stream) {
    if (check_view(x, "unet_view_materialize") || check_dims(x, n, h, w, "unet_view_materialize")) return -1;
    UNET_CHECK_ARG(out, "unet_view_materialize: null output");
    const DView v = make_dview(*x);
    const bool vec = view_vec(x);
    const int64_t work = (int64_t)n * h * w * (vec ? v.C / 4 : v.C);
    hipStream_t st = as_stream(stream);
    const int grid = grid_for(work);
    UNET_DW_DISPATCH(view_materialize_kernel, grid, v, n, h, w, out);
    UNET_CHECK_LAUNCH("unet_view_materialize");
    return 0;
}

extern "C" int unet_dwconv3x3_bwd_data(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                                       const float* dy, float* dx0, float* dx1, unet_stream_t stream) {
    if (check_view(x, "unet_dwconv3x3_bwd_data") || check_dims(x, n, h, w, "unet_dwconv3x3_bwd_data")) return -1;
    UNET_CHECK_ARG(dw_kernel && dy && dx0, "unet_dwconv3x3_bwd_data: null pointer");
    UNET_CHECK_ARG(x->mode != UNET_VIEW_CONCAT || dx1, "unet_dwconv3x3_bwd_data: CONCAT view needs dx1");
    const DView v = make_dview(*x);
    const bool vec = view_vec(x);
    if (vec && dw_tiled_ok(v.C))
        return dw_tiled_bwd_data(v, x->mode, x->drop_rate > 0.f, n, h, w, dw_kernel, dy, dx0, dx1,
                                 as_stream(stream));
    const int64_t work = (int64_t)n * h * w * (vec ? v.C / 4 : v.C);
    hipStream_t st = as_stream(stream);
    const int grid = grid_for(work);
    UNET_DW_DISPATCH(dw_bwd_data_kernel, grid, v, n, h, w, dw_kernel, dy, dx0, dx1);
    UNET_CHECK_LAUNCH("unet_dwconv3x3_bwd_data");
    return 0;
}

extern "C" int unet_dwconv3x3_bwd_data_bnstats_slabs(const unet_view* x, int n, int h, int w) {
    if (!x || (x->mode != UNET_VIEW_POOL_BNRELU && x->mode != UNET_VIEW_BNRELU) || n <= 0 || h <= 0 || w <= 0)
        return 0;
    if (!view_vec(x) || !dw_tiled_ok(x->c0)) return 0;
    return (int)dw_tiled_ntiles(n, h, w, x->c0);
}

extern "C" int unet_dwconv3x3_bwd_data_bnstats(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                                               const float* dy, float* dx0, const float* mean, const float* rstd,
                                               float* bn_partials, unet_stream_t stream) {
    const char* op = "unet_dwconv3x3_bwd_data_bnstats";
    if (check_view(x, op) || check_dims(x, n, h, w, op)) return -1;
    UNET_CHECK_ARG(dw_kernel && dy && dx0 && bn_partials, "%s: null pointer", op);
    UNET_CHECK_ARG(unet_dwconv3x3_bwd_data_bnstats_slabs(x, n, h, w) > 0,
                   "%s: needs a POOL_BNRELU or BNRELU view with channels %% 4 == 0 (tiled path)", op);
    UNET_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "%s: mean and rstd go together", op);
    const DView v = make_dview(*x);
    return dw_tiled_bwd_data_bnstats(v, x->mode, x->drop_rate > 0.f, n, h, w, dw_kernel, dy, dx0, mean, rstd, bn_partials,
                                     as_stream(stream));
}

extern "C" int unet_dwconv3x3_bwd_data_bnstats_dwf(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                                                   const float* dy, float* dx0, const float* mean, const float* rstd,
                                                   float* bn_partials, float* dw_partials, unet_stream_t stream) {
    const char* op = "unet_dwconv3x3_bwd_data_bnstats_dwf";
    if (check_view(x, op) || check_dims(x, n, h, w, op)) return -1;
    UNET_CHECK_ARG(dw_kernel && dy && dx0 && bn_partials && dw_partials, "%s: null pointer", op);
    UNET_CHECK_ARG(x->mode == UNET_VIEW_BNRELU && x->drop_rate == 0.f && unet_dwconv3x3_bwd_data_bnstats_slabs(x, n, h, w) > 0,
                   "%s: needs a BNRELU view without dropout, channels %% 4 == 0 (tiled path)", op);
    UNET_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "%s: mean and rstd go together", op);
    UNET_CHECK_ARG((uintptr_t)dw_partials % 16 == 0, "%s: dw_partials must be 16-B aligned", op);
    const DView v = make_dview(*x);
    return dw_tiled_bwd_data_bnstats(v, x->mode, false, n, h, w, dw_kernel, dy, dx0, mean, rstd, bn_partials,
                                     as_stream(stream), dw_partials);
}

extern "C" int unet_reduce_slabs(float* slabs, int S, int64_t len, float* out, unet_stream_t stream) {
    UNET_CHECK_ARG(slabs && out && S > 0 && len > 0, "unet_reduce_slabs: bad arguments");
    return reduce_slabs(slabs, S, len, out, len, len, as_stream(stream));
}

extern "C" size_t unet_dwconv3x3_bwd_filter_workspace(int n, int h, int w, int c) {
    if (n <= 0 || h <= 0 || w <= 0 || c <= 0) return 0;
    if (dw_tiled_ok(c)) return align_up(dw_tiled_filter_partials(n, h, w, c) * sizeof(float), 256);
    FilterPlan fp = filter_plan(n, h, w, c);
    return align_up((size_t)fp.chunks * 9 * c * sizeof(float), 256);
}

extern "C" int unet_dwconv3x3_bwd_filter(const unet_view* x, int n, int h, int w, const float* dy,
                                         float* d_dw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream) {
    if (check_view(x, "unet_dwconv3x3_bwd_filter") || check_dims(x, n, h, w, "unet_dwconv3x3_bwd_filter"))
        return -1;
    UNET_CHECK_ARG(dy && d_dw_kernel, "unet_dwconv3x3_bwd_filter: null pointer");
    const DView v = make_dview(*x);
    const size_t need = unet_dwconv3x3_bwd_filter_workspace(n, h, w, v.C);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_dwconv3x3_bwd_filter: workspace %zu < %zu", ws_bytes, need);
    const bool vec = view_vec(x);
    if (vec && dw_tiled_ok(v.C)) {
        int S = 0;
        float* part = static_cast<float*>(ws);
        int rc = dw_tiled_bwd_filter(v, x->mode, x->drop_rate > 0.f, n, h, w, dy, part, &S, as_stream(stream));
        if (rc) return rc;
        return reduce_slabs(part, S, (int64_t)9 * v.C, d_dw_kernel, (int64_t)9 * v.C, (int64_t)9 * v.C,
                            as_stream(stream));
    }
    FilterPlan fp = filter_plan(n, h, w, v.C);
    hipStream_t st = as_stream(stream);
    dim3 grid(fp.ctiles, (unsigned)fp.chunks);
    float* part = static_cast<float*>(ws);
    UNET_DW_DISPATCH(dw_bwd_filter_kernel, grid, v, n, h, w, dy, part, fp.ppc);
    UNET_CHECK_LAUNCH("unet_dwconv3x3_bwd_filter");
    return reduce_slabs(part, (int)fp.chunks, (int64_t)9 * v.C, d_dw_kernel, (int64_t)9 * v.C, (int64_t)9 * v.C,
                        st);
}
