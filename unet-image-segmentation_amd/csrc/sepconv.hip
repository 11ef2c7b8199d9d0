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
#include "sepconv.h"

namespace unet {

namespace {
using namespace sep;
constexpr int LR = BK + 4;                // LDS row stride (floats) of the A tile (conflict-free fragments)
constexpr int XLR = BK;                   // halo pixel stride: lane-linear, conflict-free b128 reads

// WN = waves along N (2 or 4); the block has 2 x WN waves, each owning a 64 x (BN / WN) piece of
// the 128 x BN output tile.  Wide tiles (BN = 256, 8 waves) give two waves per SIMD, so one wave's
// halo / depthwise work overlaps the other's MFMAs.
// waves per SIMD the register budget is sized for (HIP's second launch-bounds argument);
// LDS allows the matching blocks per CU
constexpr int sep_min_waves(int BN, int WN) { return WN == 2 ? (BN == 64 ? 3 : 2) : (BN == 128 ? 4 : 2); }

template <int MODE, bool DROP, int EPI, int BN, int WN, bool WRITE_Y>
__global__ __launch_bounds__(128 * WN, sep_min_waves(BN, WN)) void sepconv_fwd_kernel(SepArgs g) {
    constexpr int NT = 128 * WN;              // threads
    constexpr int LB = BN + 4;
    constexpr int TN = BN / (32 * WN);        // 32-column MFMA tiles per wave
    constexpr int NQ = BN / 4;
    constexpr int BQ = BN * (BK / 4) / NT;    // B float4 per thread per stage
    constexpr int NH = HHp * HWp * (BK / 4);  // halo float4 per stage (720)
    constexpr int HR = (NH + NT - 1) / NT;    // per thread
    constexpr int RPT = 512 / NT;             // depthwise output rows per thread (2 or 1)
    static_assert(TN >= 1 && BQ >= 1, "tile shape");
    constexpr int XS = HHp * HWp * XLR;       // floats of the (single) halo buffer
    // Pipeline (one barrier per k-stage): while the MFMAs consume A/B of stage kt, the same
    // waves evaluate the depthwise taps of stage kt+1 (halo already in LDS) and the global
    // loads of halo kt+2 / B kt+1 are in flight.
    __shared__ __attribute__((aligned(16))) float Xs[XS];
    __shared__ __attribute__((aligned(16))) float Ks[2][9 * BK];
    __shared__ __attribute__((aligned(16))) float As[2][128 * LR];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * LB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
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

    float4 rb[BQ];
    const int bq_k = tid / NQ, bq_n = tid % NQ;  // n-contiguous B: k-row, n-quad
    // Halo geometry is fixed per thread across k-stages: element e = tid + 256 j is pixel e/4 of
    // the 10x18 halo and channel quad e%4 = tid%4 of the stage.  lp = logical pixel index (-1 if
    // outside the image or past the halo), sp = first source pixel (the 2x2 window for POOL).
    // Loads are issued unconditionally from clamped addresses and masked / transformed only when
    // the registers are written to LDS, so no load is waited for before the MFMAs of the stage.
    constexpr int NP = MODE == UNET_VIEW_POOL_BNRELU ? 4 : 1;  // raw loads per halo element
    const int hq = tid & 3;
    int lp[HR], sp[HR];
#pragma unroll
    for (int j = 0; j < HR; ++j) {
        const int e = tid + NT * j;
        const int pix = e >> 2, r = pix / HWp, cc = pix - r * HWp;
        const int hh = h0 - 1 + r, ww = w0 - 1 + cc;
        const bool ok = e < NH && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
        lp[j] = ok ? (n * g.H + hh) * g.W + ww : -1;
        if constexpr (MODE == UNET_VIEW_POOL_BNRELU)
            sp[j] = ok ? (n * 2 * g.H + 2 * hh) * (2 * g.W) + 2 * ww : 0;
        else
            sp[j] = ok ? lp[j] : 0;
    }
    struct HaloRegs {
        float4 x[HR][NP];  // raw halo values in flight
        float4 sc, sh;     // BN affine of this thread's channel quad
        float4 t;          // depthwise taps (threads < 36)
        int c;             // channel of this thread's quad for the staged k0
        bool bn;
    };
    auto load_halo = [&](HaloRegs& R, int k0) {
        const int c = k0 + 4 * hq;
        R.c = c;
        const bool cok = c < Cin;
        const float* src = g.x.src0;
        int cs = g.x.c0, ci = cok ? c : 0;
        const float* scp = g.x.sc0;
        const float* shp = g.x.sh0;
        bool hbn = MODE == UNET_VIEW_BNRELU || MODE == UNET_VIEW_POOL_BNRELU;
        if constexpr (MODE == UNET_VIEW_CONCAT) {
            if (ci >= g.x.c0) {
                src = g.x.src1;
                cs = g.x.c1;
                ci -= g.x.c0;
                scp = g.x.sc1;
                shp = g.x.sh1;
                hbn = true;
            }
        }
        R.bn = hbn;
        if constexpr (MODE != UNET_VIEW_PLAIN) {
            R.sc = hbn ? ld4(scp + ci) : f4(1.f);
            R.sh = hbn ? ld4(shp + ci) : f4(0.f);
        }
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const float* b = src + (sp[j] * cs + ci);
            R.x[j][0] = ld4(b);
            if constexpr (NP == 4) {
                const int rs = 2 * g.W * cs;
                R.x[j][1] = ld4(b + cs);
                R.x[j][2] = ld4(b + rs);
                R.x[j][3] = ld4(b + rs + cs);
            }
        }
        // depthwise taps of the stage: 9 x BK floats = 36 float4, tap-major
        const int tq = tid < 9 * (BK / 4) ? tid : 0;
        const int tp = tq / (BK / 4), c2 = k0 + 4 * (tq % (BK / 4));
        R.t = ld4(g.dk + tp * Cin + (c2 < Cin ? c2 : 0));
    };
    auto store_halo = [&](const HaloRegs& R, int buf) {
        const int hc = R.c;
        const bool cok = hc < Cin;
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const int e = tid + NT * j;
            float4 v = R.x[j][0];
            if constexpr (NP == 4) {
                v = fma4(v, R.sc, R.sh);
                v = max4(v, fma4(R.x[j][1], R.sc, R.sh));
                v = max4(v, fma4(R.x[j][2], R.sc, R.sh));
                v = max4(v, fma4(R.x[j][3], R.sc, R.sh));
                v = relu4(v);
            } else if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (R.bn) v = bnrelu4(v, R.sc, R.sh);
            }
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)(lp[j] < 0 ? 0 : lp[j]) * C + hc;
                v = mul4(v, drop_mult4(g.x.seed, i, g.x.rate, g.x.inv_keep));
            }
            if (lp[j] < 0 || !cok) v = f4(0.f);
            if (e < NH) *reinterpret_cast<float4*>(&Xs[4 * e]) = v;
        }
        if (tid < 9 * (BK / 4)) {
            const int c2 = hc - 4 * hq + 4 * (tid % (BK / 4));  // k0 + quad of this tap slot
            *reinterpret_cast<float4*>(&Ks[buf][4 * tid]) = c2 < Cin ? R.t : f4(0.f);
        }
    };
    HaloRegs hr;
    bool bok[BQ];
    auto load_b = [&](int k0) {
#pragma unroll
        for (int r = 0; r < BQ; ++r) {
            const int kk = k0 + bq_k + (NT / NQ) * r, nn = n0 + 4 * bq_n;
            bok[r] = kk < Cin && nn < g.Cout;
            rb[r] = ld4(g.pk + (bok[r] ? (int64_t)kk * g.Cout + nn : 0));
        }
    };
    auto store_b = [&](int buf) {
#pragma unroll
        for (int r = 0; r < BQ; ++r)
            *reinterpret_cast<float4*>(&Bs[buf][(bq_k + (NT / NQ) * r) * LB + 4 * bq_n]) = bok[r] ? rb[r] : f4(0.f);
    };
    // depthwise taps from the staged halo into the A tile: each thread evaluates one channel quad
    // of RPT vertically adjacent pixels ((RPT + 2) x 3 LDS reads for RPT outputs)
    const int dq = tid & 3;
    const int dc = (tid >> 2) & 15, dr = RPT * (tid >> 6);
    float4 ya[RPT];  // depthwise outputs of the last dw_stage (stored to y at the end of the iteration)
    auto dw_stage = [&](int buf) {
        const float* X = Xs;
        const float* Kt = Ks[buf];
        float4 a[RPT];
#pragma unroll
        for (int o = 0; o < RPT; ++o) a[o] = f4(0.f);
#pragma unroll
        for (int i = 0; i < RPT + 2; ++i)
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                const float4 xv = *reinterpret_cast<const float4*>(&X[((dr + i) * HWp + dc + jj) * XLR + 4 * dq]);
#pragma unroll
                for (int o = 0; o < RPT; ++o)
                    if (i - o >= 0 && i - o < 3)
                        a[o] = fma4(xv, *reinterpret_cast<const float4*>(&Kt[((i - o) * 3 + jj) * BK + 4 * dq]), a[o]);
            }
#pragma unroll
        for (int o = 0; o < RPT; ++o) {
            *reinterpret_cast<float4*>(&As[buf][((dr + o) * TW + dc) * LR + 4 * dq]) = a[o];
            ya[o] = a[o];
        }
    };
    auto store_y = [&](int k0) {
        if constexpr (WRITE_Y) {
            const int c = k0 + 4 * dq;
            if (blockIdx.y == 0 && c < Cin) {
                float* yp = g.y + ((int64_t)(n * g.H + h0 + dr) * g.W + w0 + dc) * Cin + c;
#pragma unroll
                for (int o = 0; o < RPT; ++o) st4(yp + (int64_t)o * g.W * Cin, ya[o]);
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

    auto mfma_kg = [&](int buf, int kg) {
        float4 af[2], bf[TN];
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
            af[tm] = *reinterpret_cast<const float4*>(&As[buf][(wm * 64 + tm * 32 + lo) * LR + kg * 8 + 4 * hi]);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const float* bp = &Bs[buf][(kg * 8 + 4 * hi) * LB + wn * (BN / WN) + tn * 32 + lo];
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
    };

    const int nk = (Cin + BK - 1) / BK;
    // Loads past the last stage are issued from clamped (valid) addresses and their LDS images
    // are never read, so the loop body is branch-free and the compiler's vmcnt counting stays
    // exact (a conditional load forces a full drain at the join).
    // Single halo buffer: dw_stage(kt+1) reads it mid-iteration, the halo of stage kt+2 is
    // written after a barrier that follows those reads (two barriers per k-stage, one LDS copy
    // of the halo -> three blocks per CU).
    {
        HaloRegs h1;  // the first two halo stages are in flight together
        load_halo(hr, 0);
        load_b(0);
        load_halo(h1, BK);
        store_halo(hr, 0);
        store_b(0);
        __syncthreads();
        dw_stage(0);
        store_y(0);
        __syncthreads();
        store_halo(h1, 1);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        load_halo(hr, (kt + 2) * BK);
        load_b((kt + 1) * BK);
        mfma_kg(buf, 0);
        dw_stage(buf ^ 1);
        __syncthreads();  // every wave is done reading the halo of stage kt+1
        mfma_kg(buf, 1);
        store_halo(hr, buf);
        store_b(buf ^ 1);
        if (kt + 1 < nk) store_y((kt + 1) * BK);
        __syncthreads();
    }

    // epilogue: GEMM row p of the tile = pixel (h0 + p/16, w0 + p%16); all 128 rows valid
    const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = n0 + wn * (BN / WN) + tn * 32 + lo;
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
            const int cl = wn * (BN / WN) + tn * 32 + lo;
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
            const int cl = wn * (BN / WN) + tn * 32 + lo;
            mean[tn] = (red[cl] + red[BN + cl]) * (1.0f / 128.0f);
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int cl = wn * (BN / WN) + tn * 32 + lo;
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
                const int cl = wn * (BN / WN) + tn * 32 + lo;
                const int col = n0 + cl;
                if (col < g.Cout)
                    g.stats[(int64_t)blockIdx.x * g.Cout + col] = make_float2(mean[tn], red[cl] + red[BN + cl]);
            }
        }
    }
}

template <int MODE, bool DROP, int BN, int WN>
void launch_tile(const SepArgs& a, bool stats, bool write_y, hipStream_t st) {
    const dim3 grid((unsigned)(a.N * (a.H / TH) * (a.W / TW)), (unsigned)cdiv(a.Cout, BN));
    constexpr int NT = 128 * WN;
    if (stats) {
        if (write_y) sepconv_fwd_kernel<MODE, DROP, E_STATS, BN, WN, true><<<grid, NT, 0, st>>>(a);
        else sepconv_fwd_kernel<MODE, DROP, E_STATS, BN, WN, false><<<grid, NT, 0, st>>>(a);
    } else {
        if (write_y) sepconv_fwd_kernel<MODE, DROP, E_STORE, BN, WN, true><<<grid, NT, 0, st>>>(a);
        else sepconv_fwd_kernel<MODE, DROP, E_STORE, BN, WN, false><<<grid, NT, 0, st>>>(a);
    }
}

template <int MODE, bool DROP>
int launch(const SepArgs& a, bool stats, bool write_y, hipStream_t st) {
    // the 256-wide, 8-wave tile when it still gives every CU (256) a block; else 128 (measured:
    // tools/bench_sepconv.py, profiles/r1i_sepconv_bn_sweep.log)
    const int64_t mt = (int64_t)a.N * (a.H / TH) * (a.W / TW);
    int bn = a.Cout <= 64 ? 64 : a.Cout <= 128 ? 128 : 256;
    if (bn == 256 && mt * cdiv(a.Cout, 256) < 256) bn = 128;
    if (bn == 64)
        launch_tile<MODE, DROP, 64, 2>(a, stats, write_y, st);
    else if (bn == 128)
        launch_tile<MODE, DROP, 128, 2>(a, stats, write_y, st);
    else
        launch_tile<MODE, DROP, 256, 4>(a, stats, write_y, st);
    UNET_CHECK_LAUNCH("unet_sepconv_fwd");
    return 0;
}

}  // namespace
}  // namespace unet

using namespace unet;

namespace {
int g_sep_schedule = UNET_SEPCONV_AUTO;
}

extern "C" int unet_sepconv_set_schedule(int schedule) {
    UNET_CHECK_ARG(schedule >= UNET_SEPCONV_AUTO && schedule <= UNET_SEPCONV_RK1, "unet_sepconv_set_schedule: bad value");
    const int old = g_sep_schedule;
    g_sep_schedule = schedule;
    return old;
}

extern "C" int unet_sepconv_fwd_supported(const unet_view* x, int n, int h, int w, int cout) {
    if (!x || n <= 0 || h <= 0 || w <= 0 || cout <= 0) return 0;
    const int C = x->c0 + (x->mode == UNET_VIEW_CONCAT ? x->c1 : 0);
    if (h % TH || w % TW || C % 4 || cout % 4) return 0;
    if (x->mode == UNET_VIEW_CONCAT && x->c0 % 4) return 0;
    const int64_t M = (int64_t)n * h * w;
    return M * C < (int64_t(1) << 31) && M * cout < (int64_t(1) << 31) &&
           (int64_t)n * h * w * C * (x->mode == UNET_VIEW_POOL_BNRELU ? 4 : 1) < (int64_t(1) << 31);
}

namespace unet {
namespace {
// zsel[n][i][j][c] = pool_sel over z's 2x2 window (2i..2i+1, 2j..2j+1), channel quads
__global__ __launch_bounds__(256) void pool_select_kernel(const float* __restrict__ z, int64_t quads, int H2, int W2,
                                                          int C, const float* __restrict__ gamma, float* __restrict__ out) {
    const int C4 = C / 4;
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < quads; e += (int64_t)gridDim.x * 256) {
        const int q = (int)(e % C4);
        const int64_t p = e / C4;  // pooled pixel (n, i, j)
        const int j = (int)(p % W2);
        const int64_t ni = p / W2;  // n * H2 + i
        const int64_t r0 = (2 * ni) * (2 * W2) + 2 * j;  // z pixel (n, 2i, 2j): rows of 2 W2 pixels
        const float* b = z + r0 * C + 4 * q;
        const float4 a = ld4(b), bb = ld4(b + C), c = ld4(b + 2 * W2 * C), d = ld4(b + 2 * W2 * C + C);
        const float4 gm = gamma ? ld4(gamma + 4 * q) : f4(0.f);
        float4 o;
        o.x = sep::pool_sel(a.x, bb.x, c.x, d.x, signbit(gm.x));
        o.y = sep::pool_sel(a.y, bb.y, c.y, d.y, signbit(gm.y));
        o.z = sep::pool_sel(a.z, bb.z, c.z, d.z, signbit(gm.z));
        o.w = sep::pool_sel(a.w, bb.w, c.w, d.w, signbit(gm.w));
        st4(out + p * C + 4 * q, o);
    }
}
}  // namespace
}  // namespace unet

extern "C" int unet_pool_select(const float* z, int n, int h, int w, int c, const float* gamma, float* out,
                                unet_stream_t stream) {
    UNET_CHECK_ARG(z && out && n > 0 && h > 0 && w > 0 && c > 0, "unet_pool_select: bad arguments");
    UNET_CHECK_ARG(h % 2 == 0 && w % 2 == 0 && c % 4 == 0, "unet_pool_select: needs even h, w and c %% 4 == 0");
    UNET_CHECK_ARG(((uintptr_t)z | (uintptr_t)out | (uintptr_t)gamma) % 16 == 0, "unet_pool_select: 16-B alignment");
    const int64_t quads = (int64_t)n * (h / 2) * (w / 2) * (c / 4);
    int64_t blocks = (quads + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    pool_select_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(z, quads, h / 2, w / 2, c, gamma, out);
    UNET_CHECK_LAUNCH("unet_pool_select");
    return 0;
}

extern "C" int unet_sepconv_fwd(const unet_view* x, int n, int h, int w, const float* dw_kernel, int cout,
                                const float* pw_kernel, const unsigned short* pw_kernel_x3, float* y, float* z,
                                float* bn_partials, float* z_pool_sel, const float* gamma, unet_stream_t stream) {
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
    if (z_pool_sel) {
        UNET_CHECK_ARG(h % 2 == 0 && w % 2 == 0 && ((uintptr_t)z_pool_sel | (uintptr_t)gamma) % 16 == 0,
                       "unet_sepconv_fwd: z_pool_sel needs even h, w and 16-B aligned buffers");
    }
    if (z_pool_sel && !(g_sep_schedule != UNET_SEPCONV_TILE && rk_supported(x->mode, a.Cin, cout))) {
        // LDS-A-tile schedule: the selection in a pass over z after the kernel
        const int rc = unet_sepconv_fwd(x, n, h, w, dw_kernel, cout, pw_kernel, pw_kernel_x3, y, z, bn_partials,
                                        nullptr, nullptr, stream);
        return rc ? rc : unet_pool_select(z, n, h, w, cout, gamma, z_pool_sel, stream);
    }
    a.zsel = z_pool_sel;
    a.gamma = gamma;
    UNET_CHECK_ARG(((uintptr_t)pw_kernel_x3 & 15) == 0, "unet_sepconv_fwd: pw_kernel_x3 must be 16-B aligned");
    a.pkx = pw_kernel_x3;
    // register-A schedule where it exists (rk_supported: BN+ReLU / concat / plain views of >= 64
    // channels, max-pool views of >= 64 inputs and <= 128 outputs) unless the LDS-A-tile schedule
    // is forced; wider max-pool views keep the LDS-A-tile kernel (its 256-wide 8-wave tile pools
    // each halo element once for all columns)
    if (g_sep_schedule != UNET_SEPCONV_TILE && rk_supported(x->mode, a.Cin, cout)) {
        // the persistent split-precision kernel for the short-K shapes (sepconv_px.hip), unless
        // the one-tile-per-block register-A kernel is forced
        if (g_sep_schedule != UNET_SEPCONV_RK1 && px_supported(a, x->mode, g_sep_schedule == UNET_SEPCONV_RK)) {
            if (launch_px(a, x->mode, drop, stats, wy, st)) return -1;
            UNET_CHECK_LAUNCH("unet_sepconv_fwd");
            return 0;
        }
        if (launch_rk(a, x->mode, drop, stats, wy, st)) return -1;
        UNET_CHECK_LAUNCH("unet_sepconv_fwd");
        return 0;
    }
    UNET_CHECK_ARG(g_sep_schedule != UNET_SEPCONV_RK, "unet_sepconv_fwd: no register-A kernel for this view / shape");
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
