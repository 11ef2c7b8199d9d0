// Fused SeparableConv2D forward (reference model/u_net.py:14-20): depthwise 3x3 -> pointwise
// 1x1 in one kernel, with the BatchNorm-statistics epilogue (u_net.py:22-23).
//
// GEMM z[M, Cout] = dw(x)[M, Cin] . P[Cin, Cout] where the A operand is never materialised in
// HBM: each 128-row M tile is an 8 x 16 pixel rectangle of one image; per 16-channel k-stage
// the block stages the 10 x 18 halo of the input VIEW (BN affine + ReLU / max-pool / concat /
// dropout applied once per staged element) into LDS, evaluates the 3x3 depthwise taps from LDS
// straight into the MFMA A tile (k-contiguous rows, stride 20 floats, conflict-free
// ds_read_b128 fragments as in gemm_rows_vec), then runs v_mfma_f32_32x32x2_f32 on it.
// In training the first N-tile block also stores y (the depthwise output), which the pointwise
// weight gradient needs; inference skips it.  Requires H % 8 == 0, W % 16 == 0, Cin % 4 == 0.
#include "view.h"

namespace unet {

namespace {

constexpr int TH = 8, TW = 16;            // pixel rectangle of one M tile
constexpr int HHp = TH + 2, HWp = TW + 2; // halo
constexpr int BK = 16;                    // channels per k-stage
constexpr int LR = BK + 4;                // LDS row stride (floats) of A / halo / k-contiguous B
enum { E_STORE = 0, E_STATS = 1 };

__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

struct SepArgs {
    DView x;
    int N, H, W, Cin, Cout;
    const float* dk;  // (3,3,Cin,1)
    const float* pk;  // (1,1,Cin,Cout): B(k, n) = pk[k*Cout + n] (n-contiguous)
    float* y;         // optional (N,H,W,Cin)
    float* z;         // (N,H,W,Cout)
    float2* stats;    // [M/128][Cout]
};

template <int MODE, bool DROP, int EPI, int BN, bool WRITE_Y>
__global__ __launch_bounds__(256) void sepconv_fwd_kernel(SepArgs g) {
    constexpr int LB = BN + 4;
    constexpr int TN = BN / 64;
    constexpr int NQ = BN / 4;
    constexpr int BQ = BN * (BK / 4) / 256;  // B float4 per thread per stage
    constexpr int NH = HHp * HWp * (BK / 4);  // halo float4 per stage (720)
    constexpr int HR = (NH + 255) / 256;      // per thread (3)
    __shared__ __attribute__((aligned(16))) float Xs[HHp * HWp * LR];
    __shared__ __attribute__((aligned(16))) float As[2][128 * LR];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * LB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lo = lane & 31, hi = lane >> 5;
    const int tiles_w = g.W / TW, tiles_h = g.H / TH;
    int t = blockIdx.x;
    const int tw = t % tiles_w;
    t /= tiles_w;
    const int th = t % tiles_h;
    const int n = t / tiles_h;
    const int h0 = th * TH, w0 = tw * TW;
    const int n0 = blockIdx.y * BN;
    const int Cin = g.Cin, C = g.x.C;

    // halo staging geometry: element e = tid + 256 j -> (pixel, quad)
    float4 rh[HR];
    float4 rb[BQ];
    float4 rk[9];
    const int dq = tid & 3;                   // dw_stage: channel quad
    const int dc = (tid >> 2) & 15, dr = 2 * (tid >> 6);  // dw_stage: pixel column, first of 2 rows
    const int bq_k = tid / NQ, bq_n = tid % NQ;  // n-contiguous B: k-row, n-quad
    auto load_stage = [&](int k0) {
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const int e = tid + 256 * j;
            float4 v = f4(0.f);
            if (e < NH) {
                const int q = e & 3, pix = e >> 2;
                const int r = pix / HWp, cc = pix - (pix / HWp) * HWp;
                const int hh = h0 - 1 + r, ww = w0 - 1 + cc;
                const int c = k0 + 4 * q;
                if (hh >= 0 && hh < g.H && ww >= 0 && ww < g.W && c < Cin) {
                    v = view_load4<MODE>(g.x, n, hh, ww, g.H, g.W, c);
                    if constexpr (DROP) {
                        const uint64_t i = ((uint64_t)((n * g.H + hh) * g.W + ww)) * C + c;
                        v.x *= drop_mult(g.x.seed, i + 0, g.x.rate, g.x.inv_keep);
                        v.y *= drop_mult(g.x.seed, i + 1, g.x.rate, g.x.inv_keep);
                        v.z *= drop_mult(g.x.seed, i + 2, g.x.rate, g.x.inv_keep);
                        v.w *= drop_mult(g.x.seed, i + 3, g.x.rate, g.x.inv_keep);
                    }
                }
            }
            rh[j] = v;
        }
#pragma unroll
        for (int r = 0; r < BQ; ++r) {
            const int kk = k0 + bq_k + (256 / NQ) * r, nn = n0 + 4 * bq_n;
            rb[r] = (kk < Cin && nn < g.Cout) ? ld4(g.pk + (int64_t)kk * g.Cout + nn) : f4(0.f);
        }
        const int c = k0 + 4 * dq;  // depthwise taps of this thread's channel quad, prefetched
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) rk[tp] = c < Cin ? ld4(g.dk + tp * Cin + c) : f4(0.f);
    };
    auto store_stage = [&](int buf) {
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const int e = tid + 256 * j;
            if (e < NH) *reinterpret_cast<float4*>(&Xs[(e >> 2) * LR + 4 * (e & 3)]) = rh[j];
        }
#pragma unroll
        for (int r = 0; r < BQ; ++r)
            *reinterpret_cast<float4*>(&Bs[buf][(bq_k + (256 / NQ) * r) * LB + 4 * bq_n]) = rb[r];
    };
    // depthwise taps from the staged halo into the A tile: each thread evaluates one channel quad
    // of two vertically adjacent pixels (4 halo rows x 3 columns of LDS reads for 2 outputs)
    auto dw_stage = [&](int k0, int buf) {
        float4 a0 = f4(0.f), a1 = f4(0.f);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                const float4 xv = *reinterpret_cast<const float4*>(&Xs[((dr + i) * HWp + dc + jj) * LR + 4 * dq]);
                if (i < 3) a0 = fma4(xv, rk[i * 3 + jj], a0);
                if (i > 0) a1 = fma4(xv, rk[(i - 1) * 3 + jj], a1);
            }
        const int p0 = dr * TW + dc;
        *reinterpret_cast<float4*>(&As[buf][p0 * LR + 4 * dq]) = a0;
        *reinterpret_cast<float4*>(&As[buf][(p0 + TW) * LR + 4 * dq]) = a1;
        if constexpr (WRITE_Y) {
            const int c = k0 + 4 * dq;
            if (blockIdx.y == 0 && c < Cin) {
                float* yp = g.y + ((int64_t)(n * g.H + h0 + dr) * g.W + w0 + dc) * Cin + c;
                st4(yp, a0);
                st4(yp + (int64_t)g.W * Cin, a1);
            }
        }
    };

    floatx16 acc[2][TN];
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

    const int nk = (Cin + BK - 1) / BK;
    load_stage(0);
    store_stage(0);
    __syncthreads();
    dw_stage(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        const bool more = kt + 1 < nk;
        if (more) load_stage((kt + 1) * BK);
#pragma unroll
        for (int kg = 0; kg < BK / 8; ++kg) {
            float4 af[2], bf[TN];
#pragma unroll
            for (int tm = 0; tm < 2; ++tm)
                af[tm] = *reinterpret_cast<const float4*>(&As[buf][(wm * 64 + tm * 32 + lo) * LR + kg * 8 + 4 * hi]);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const float* bp = &Bs[buf][(kg * 8 + 4 * hi) * LB + wn * (BN / 2) + tn * 32 + lo];
                bf[tn] = make_float4(bp[0], bp[LB], bp[2 * LB], bp[3 * LB]);
            }
#pragma unroll
            for (int tm = 0; tm < 2; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].x, bf[tn].x, acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].y, bf[tn].y, acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].z, bf[tn].z, acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].w, bf[tn].w, acc[tm][tn], 0, 0, 0);
                }
        }
        if (more) store_stage(buf ^ 1);  // Xs was last read by dw_stage(kt), before the last barrier
        __syncthreads();
        if (more) dw_stage((kt + 1) * BK, buf ^ 1);
        __syncthreads();
    }

    // epilogue: GEMM row p of the tile = pixel (h0 + p/16, w0 + p%16); all 128 rows valid
    const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = n0 + wn * (BN / 2) + tn * 32 + lo;
            if (col >= g.Cout) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int p = wm * 64 + tm * 32 + acc_row(r, hi);
                g.z[(mbase + (int64_t)(p >> 4) * g.W + (p & 15)) * g.Cout + col] = acc[tm][tn][r];
            }
        }
    if constexpr (EPI == E_STATS) {
        float* red = &As[0][0];
        float mean[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int cl = wn * (BN / 2) + tn * 32 + lo;
            float s = 0.f;
#pragma unroll
            for (int tm = 0; tm < 2; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r) s += acc[tm][tn][r];
            s += __shfl_xor(s, 32, 64);
            if (hi == 0) red[wm * BN + cl] = s;
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int cl = wn * (BN / 2) + tn * 32 + lo;
            mean[tn] = (red[cl] + red[BN + cl]) * (1.0f / 128.0f);
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int cl = wn * (BN / 2) + tn * 32 + lo;
            float q = 0.f;
#pragma unroll
            for (int tm = 0; tm < 2; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float d = acc[tm][tn][r] - mean[tn];
                    q = fmaf(d, d, q);
                }
            q += __shfl_xor(q, 32, 64);
            if (hi == 0) red[wm * BN + cl] = q;
        }
        __syncthreads();
        if (wm == 0 && hi == 0) {
            // stats row index = the tile's M-order index: tiles are 128-row units of M only when
            // the tile is a full 128-pixel run; with 8x16 rectangles the partial is indexed by
            // tile id (bn_finalize only needs 128-row counts, which all tiles have).
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int cl = wn * (BN / 2) + tn * 32 + lo;
                const int col = n0 + cl;
                if (col < g.Cout)
                    g.stats[(int64_t)blockIdx.x * g.Cout + col] = make_float2(mean[tn], red[cl] + red[BN + cl]);
            }
        }
    }
}

template <int MODE, bool DROP>
int launch(const SepArgs& a, bool stats, bool write_y, hipStream_t st) {
    const unsigned tiles = (unsigned)(a.N * (a.H / TH) * (a.W / TW));
#define UNET_SEP(BN_)                                                                                        \
    {                                                                                                        \
        dim3 grid(tiles, (unsigned)cdiv(a.Cout, BN_));                                                       \
        if (stats) {                                                                                         \
            if (write_y) sepconv_fwd_kernel<MODE, DROP, E_STATS, BN_, true><<<grid, 256, 0, st>>>(a);        \
            else sepconv_fwd_kernel<MODE, DROP, E_STATS, BN_, false><<<grid, 256, 0, st>>>(a);               \
        } else {                                                                                             \
            if (write_y) sepconv_fwd_kernel<MODE, DROP, E_STORE, BN_, true><<<grid, 256, 0, st>>>(a);        \
            else sepconv_fwd_kernel<MODE, DROP, E_STORE, BN_, false><<<grid, 256, 0, st>>>(a);               \
        }                                                                                                    \
    }
    if (a.Cout <= 64)
        UNET_SEP(64)
    else
        UNET_SEP(128)
#undef UNET_SEP
    UNET_CHECK_LAUNCH("unet_sepconv_fwd");
    return 0;
}

}  // namespace
}  // namespace unet

using namespace unet;

extern "C" int unet_sepconv_fwd_supported(const unet_view* x, int n, int h, int w, int cout) {
    if (!x || n <= 0 || h <= 0 || w <= 0 || cout <= 0) return 0;
    const int C = x->c0 + (x->mode == UNET_VIEW_CONCAT ? x->c1 : 0);
    if (h % TH || w % TW || C % 4 || cout % 4) return 0;
    if (x->mode == UNET_VIEW_CONCAT && x->c0 % 4) return 0;
    const int64_t M = (int64_t)n * h * w;
    return M * C < (int64_t(1) << 31) && M * cout < (int64_t(1) << 31) &&
           (int64_t)n * h * w * C * (x->mode == UNET_VIEW_POOL_BNRELU ? 4 : 1) < (int64_t(1) << 31);
}

extern "C" int unet_sepconv_fwd(const unet_view* x, int n, int h, int w, const float* dw_kernel, int cout,
                                const float* pw_kernel, float* y, float* z, float* bn_partials,
                                unet_stream_t stream) {
    if (check_view(x, "unet_sepconv_fwd")) return -1;
    UNET_CHECK_ARG(unet_sepconv_fwd_supported(x, n, h, w, cout),
                   "unet_sepconv_fwd: unsupported shape (needs h%%8==0, w%%16==0, channels%%4==0)");
    UNET_CHECK_ARG(dw_kernel && pw_kernel && z, "unet_sepconv_fwd: null pointer");
    SepArgs a{};
    a.x = make_dview(*x);
    a.N = n;
    a.H = h;
    a.W = w;
    a.Cin = a.x.C;
    a.Cout = cout;
    a.dk = dw_kernel;
    a.pk = pw_kernel;
    a.y = y;
    a.z = z;
    a.stats = reinterpret_cast<float2*>(bn_partials);
    const bool stats = bn_partials != nullptr, wy = y != nullptr, drop = x->drop_rate > 0.f;
    hipStream_t st = as_stream(stream);
    switch (x->mode) {
        case UNET_VIEW_PLAIN:
            return drop ? launch<UNET_VIEW_PLAIN, true>(a, stats, wy, st) : launch<UNET_VIEW_PLAIN, false>(a, stats, wy, st);
        case UNET_VIEW_BNRELU:
            return drop ? launch<UNET_VIEW_BNRELU, true>(a, stats, wy, st)
                        : launch<UNET_VIEW_BNRELU, false>(a, stats, wy, st);
        case UNET_VIEW_POOL_BNRELU:
            return drop ? launch<UNET_VIEW_POOL_BNRELU, true>(a, stats, wy, st)
                        : launch<UNET_VIEW_POOL_BNRELU, false>(a, stats, wy, st);
        default:
            return drop ? launch<UNET_VIEW_CONCAT, true>(a, stats, wy, st)
                        : launch<UNET_VIEW_CONCAT, false>(a, stats, wy, st);
    }
}
