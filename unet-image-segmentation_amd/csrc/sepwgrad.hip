// Weight gradients of a 64 -> 64 SeparableConv2D (reference model/u_net.py:14-20; the pixel
// reductions of Keras' implicit backward, scripts/train.py:308) in ONE pass that never reads the
// depthwise output y:
//
//   d_pw[ci][co] = sum_px y[px][ci] dz[px][co]          y = depthwise3x3(x), recomputed here
//   d_dw[t][ci]  = sum_px x[px + off(t)][ci] dy[px][ci]  (the 3x3 taps y is formed from)
//
// x is the block's input VIEW (BN affine + ReLU / concat / dropout on load, zero padding).  These
// are the 256 x 256 level's conv blocks (enc1_block2, dec1_block2), HBM-bound: the separate route
// (unet_pointwise_bwd_filter over a stored y, then unet_dwconv3x3_bwd_filter over (x, dy)) moves
// y twice (forward store + read) and x once more.  Here the forward keeps no y, and the backward
// streams x, dz and dy once: 768 B per pixel.
//
// One block (8 waves) per CU walks a contiguous run of 8 x 16 pixel tiles.  Per tile:
//   * the 10 x 18 halo of the view (64 channels) and the dz tile -> LDS (register staged: the next
//     tile's loads are in flight while this one computes); each thread's dy quads -> registers
//     (loaded once this tile's filter-gradient FMAs have consumed the previous ones);
//   * every thread evaluates 4 (pixel, 4-channel) quads of y from 9 conflict-free ds_read_b128
//     taps with the forward's k-ordered fmaf chain (y bitwise equal to unet_sepconv_fwd's) into
//     the LDS y tile, and accumulates the depthwise filter gradient from the same taps;
//   * wave w runs v_mfma_f32_32x32x2_f32 for its 32 x 32 (ci, co) quarter over half the tile's
//     pixels (A = y^T, B = dz: one conflict-free ds_read_b32 each per MFMA).
// The two pixel halves of each quarter and the 32 threads per channel quad of the filter gradient
// are combined in fixed order; one slab per block, reduced by reduce_slabs in fixed order.
#include "common.h"
#include "view.h"

namespace unet {
namespace {

constexpr int TH = 8, TW = 16, HWp = TW + 2, HPIX = (TH + 2) * HWp;  // 180 halo pixels
constexpr int CI = 64, CO = 64;                                       // channels
constexpr int NT = 512;                                               // threads
constexpr int NHQ = HPIX * (CI / 4);                                  // halo float4 (2880)
constexpr int HR = (NHQ + NT - 1) / NT;                               // per thread (6)
constexpr int DQ = 128 * CO / 4 / NT;                                 // dz float4 per thread (4)
constexpr int LDS_HALO = HPIX * CI, LDS_YT = 128 * CI, LDS_DZ = 128 * CO;
constexpr int LDS_SIZE = LDS_HALO + LDS_YT + LDS_DZ;                  // 110 KB
static_assert(2 * 64 * 64 <= LDS_SIZE && 9 * 32 * 16 * 4 <= LDS_SIZE, "epilogue scratch");

__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

struct SwArgs {
    DView x;
    int N, H, W;
    const float* dk;  // (3,3,64,1)
    const float* dy;  // (M, 64)
    const float* dz;  // (M, 64)
    float* pw_slab;   // [S][64][64]
    float* dw_slab;   // [S][9][64]
    int tiles, tps;   // pixel tiles, tiles per block
};

template <int MODE, bool DROP>
__global__ __launch_bounds__(NT, 1) void sepconv_wgrad64_kernel(SwArgs g) {
    __shared__ __attribute__((aligned(16))) float smem[LDS_SIZE];
    float* Xs = smem;
    float* Ys = smem + LDS_HALO;
    float* Zs = smem + LDS_HALO + LDS_YT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    const int t_begin = blockIdx.x * g.tps;
    const int t_end = t_begin + g.tps < g.tiles ? t_begin + g.tps : g.tiles;
    const int tiles_w = g.W / TW, tiles_h = g.H / TH;
    const int C = g.x.C;

    // this thread's channel quad (halo staging, y and filter-gradient quads alike)
    const int cq = tid & 15, ci = 4 * cq;
    float4 kt[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) kt[t] = ld4(g.dk + t * CI + ci);
    const float* src = g.x.src0;
    int cs = g.x.c0, cc = ci;
    const float* scp = g.x.sc0;
    const float* shp = g.x.sh0;
    bool bn = MODE == UNET_VIEW_BNRELU;
    if constexpr (MODE == UNET_VIEW_CONCAT) {
        if (cc >= g.x.c0) {
            src = g.x.src1;
            cs = g.x.c1;
            cc -= g.x.c0;
            scp = g.x.sc1;
            shp = g.x.sh1;
            bn = true;
        }
    }
    float4 hsc = f4(1.f), hsh = f4(0.f);
    if constexpr (MODE != UNET_VIEW_PLAIN) {
        if (bn) {
            hsc = ld4(scp + cc);
            hsh = ld4(shp + cc);
        }
    }

    float4 hx[HR], rz[DQ], rdy[4];
    int lp[HR];
    auto load = [&](int T) {
        const int tw = T % tiles_w, r0 = T / tiles_w;
        const int h0 = (r0 % tiles_h) * TH, n = r0 / tiles_h, w0 = tw * TW;
#pragma unroll
        for (int k = 0; k < HR; ++k) {
            const int e = tid + NT * k;
            const int pix = e >> 4, r = pix / HWp, c = pix - r * HWp;
            const int hh = h0 - 1 + r, ww = w0 - 1 + c;
            const bool ok = e < NHQ && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
            lp[k] = ok ? (n * g.H + hh) * g.W + ww : -1;
            hx[k] = ld4(src + ((int64_t)(ok ? lp[k] : 0) * cs + cc));
        }
        const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
        for (int k = 0; k < DQ; ++k) {  // dz tile: element e = pixel e >> 4, quad e & 15
            const int e = tid + NT * k, p = e >> 4, q = e & 15;
            rz[k] = ld4(g.dz + (mbase + (int64_t)(p >> 4) * g.W + (p & 15)) * CO + 4 * q);
        }
    };
    auto load_dy = [&](int T) {  // dy of this thread's quads: pixel (tid >> 4) + 32 k
        const int tw = T % tiles_w, r0 = T / tiles_w;
        const int h0 = (r0 % tiles_h) * TH, n = r0 / tiles_h, w0 = tw * TW;
        const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = (tid >> 4) + 32 * k;
            rdy[k] = ld4(g.dy + (mbase + (int64_t)(p >> 4) * g.W + (p & 15)) * CI + ci);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int k = 0; k < HR; ++k) {
            const int e = tid + NT * k;
            float4 v = hx[k];
            if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (bn) v = bnrelu4(v, hsc, hsh);
            }
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)(lp[k] < 0 ? 0 : lp[k]) * C + ci;
                v = mul4(v, drop_mult4(g.x.seed, i, g.x.rate, g.x.inv_keep));
            }
            if (lp[k] < 0) v = f4(0.f);
            if (e < NHQ) *reinterpret_cast<float4*>(&Xs[(e >> 4) * CI + 4 * (e & 15)]) = v;
        }
#pragma unroll
        for (int k = 0; k < DQ; ++k) {
            const int e = tid + NT * k;
            *reinterpret_cast<float4*>(&Zs[(e >> 4) * CO + 4 * (e & 15)]) = rz[k];
        }
    };

    // MFMA quarter of this wave: ci rows 32 (w & 1) .., co columns 32 ((w >> 1) & 1) .., pixels
    // 64 (w >> 2) .. +63 of the tile (32 k-steps of 2)
    const int wci = 32 * (wave & 1), wco = 32 * ((wave >> 1) & 1), wpx = 64 * (wave >> 2);
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float4 dwa[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) dwa[t] = f4(0.f);

    if (t_begin < t_end) {
        load(t_begin);
        load_dy(t_begin);
    }
    for (int T = t_begin; T < t_end; ++T) {
        store();
        __syncthreads();
        load(T + 1 < t_end ? T + 1 : T);  // next tile in flight (past the end: a valid, unused tile)
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {  // (not unrolled: 9 taps in flight, not 36)
            const int p = (tid >> 4) + 32 * k, pr = p >> 4, pc = p & 15;
            const float4 dq = rdy[0];  // static register indexing: rotate the dy quads
            rdy[0] = rdy[1];
            rdy[1] = rdy[2];
            rdy[2] = rdy[3];
            float4 y = f4(0.f);
#pragma unroll
            for (int dy_ = 0; dy_ < 3; ++dy_)
#pragma unroll
                for (int dx_ = 0; dx_ < 3; ++dx_) {
                    const float4 xv = *reinterpret_cast<const float4*>(&Xs[((pr + dy_) * HWp + pc + dx_) * CI + ci]);
                    y = fma4(xv, kt[dy_ * 3 + dx_], y);
                    dwa[dy_ * 3 + dx_] = fma4(xv, dq, dwa[dy_ * 3 + dx_]);
                }
            *reinterpret_cast<float4*>(&Ys[p * CI + ci]) = y;
        }
        load_dy(T + 1 < t_end ? T + 1 : T);  // its latency hides behind the MFMA phase
        __syncthreads();
#pragma unroll 4
        for (int s = 0; s < 32; ++s) {
            const int p = wpx + 2 * s + hi;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ys[p * CI + wci + lo], Zs[p * CO + wco + lo], acc, 0, 0, 0);
        }
        __syncthreads();
    }

    // pointwise slab [ci][co]: the two pixel halves of each (ci, co) quarter, fixed order
    float* E = smem;  // [2 pixel halves][64 ci][64 co]
#pragma unroll
    for (int r = 0; r < 16; ++r) E[((wave >> 2) * 64 + wci + acc_row(r, hi)) * CO + wco + lo] = acc[r];
    __syncthreads();
    float* pw = g.pw_slab + (int64_t)blockIdx.x * CI * CO;
    for (int e = tid; e < CI * CO / 4; e += NT) {
        const float4 a = *reinterpret_cast<const float4*>(&E[4 * e]);
        const float4 b = *reinterpret_cast<const float4*>(&E[CI * CO + 4 * e]);
        st4(pw + 4 * e, add4(a, b));
    }
    __syncthreads();
    // depthwise slab [t][ci]: the 32 threads of each channel quad, fixed-order tree
    float4* D = reinterpret_cast<float4*>(smem);  // [9][32 pixel rows][16 quads]
#pragma unroll
    for (int t = 0; t < 9; ++t) D[(t * 32 + (tid >> 4)) * 16 + cq] = dwa[t];
    __syncthreads();
    for (int o = 16; o > 0; o >>= 1) {
        for (int e = tid; e < 9 * o * 16; e += NT) {
            const int t = e / (o * 16), rr = (e / 16) % o, q = e % 16;
            D[(t * 32 + rr) * 16 + q] = add4(D[(t * 32 + rr) * 16 + q], D[(t * 32 + rr + o) * 16 + q]);
        }
        __syncthreads();
    }
    float* dws = g.dw_slab + (int64_t)blockIdx.x * 9 * CI;
    if (tid < 9 * 16) st4(dws + (tid / 16) * CI + 4 * (tid % 16), D[(tid / 16) * 32 * 16 + (tid % 16)]);
}

int resident_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

struct SwPlan {
    int tiles, S, tps;
};
SwPlan sw_plan(int n, int h, int w) {
    SwPlan p;
    p.tiles = n * (h / TH) * (w / TW);
    const int cus = resident_cus();
    p.tps = (int)cdiv(p.tiles, cus);  // one block per CU (110 KB of LDS)
    p.S = (int)cdiv(p.tiles, p.tps);
    return p;
}

template <int MODE, bool DROP>
void launch_sw(const SwArgs& a, int blocks, hipStream_t st) {
    sepconv_wgrad64_kernel<MODE, DROP><<<blocks, NT, 0, st>>>(a);
}

}  // namespace
}  // namespace unet

using namespace unet;

extern "C" int unet_sepconv_bwd_filter_supported(const unet_view* x, int n, int h, int w, int cout) {
    if (!x || n <= 0 || h <= 0 || w <= 0 || cout != CO) return 0;
    if (x->mode != UNET_VIEW_PLAIN && x->mode != UNET_VIEW_BNRELU && x->mode != UNET_VIEW_CONCAT) return 0;
    const int C = x->c0 + (x->mode == UNET_VIEW_CONCAT ? x->c1 : 0);
    if (C != CI || h % TH || w % TW) return 0;
    if (x->mode == UNET_VIEW_CONCAT && x->c0 % 4) return 0;
    return (int64_t)n * h * w * CI < (int64_t(1) << 31);
}

extern "C" size_t unet_sepconv_bwd_filter_workspace(int n, int h, int w, int cin, int cout) {
    if (n <= 0 || h <= 0 || w <= 0 || cin != CI || cout != CO || h % TH || w % TW) return 0;
    const SwPlan p = sw_plan(n, h, w);
    return align_up((size_t)p.S * CI * CO * sizeof(float), 256) + align_up((size_t)p.S * 9 * CI * sizeof(float), 256);
}

extern "C" int unet_sepconv_bwd_filter(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                                       const float* dy, const float* dz, int cout, float* d_dw_kernel,
                                       float* d_pw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream) {
    if (check_view(x, "unet_sepconv_bwd_filter")) return -1;
    UNET_CHECK_ARG(unet_sepconv_bwd_filter_supported(x, n, h, w, cout),
                   "unet_sepconv_bwd_filter: unsupported shape (needs 64 input and output channels, a PLAIN / "
                   "BNRELU / CONCAT view, h %% 8 == 0, w %% 16 == 0)");
    UNET_CHECK_ARG(dw_kernel && dy && dz && d_dw_kernel && d_pw_kernel, "unet_sepconv_bwd_filter: null pointer");
    UNET_CHECK_ARG(((uintptr_t)dy | (uintptr_t)dz | (uintptr_t)dw_kernel | (uintptr_t)x->src0 |
                    (uintptr_t)(x->src1 ? x->src1 : x->src0)) % 16 == 0,
                   "unet_sepconv_bwd_filter: operands must be 16-B aligned");
    const size_t need = unet_sepconv_bwd_filter_workspace(n, h, w, CI, CO);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_sepconv_bwd_filter: workspace %zu < %zu", ws_bytes, need);
    const SwPlan p = sw_plan(n, h, w);
    SwArgs a{};
    a.x = make_dview(*x);
    a.N = n;
    a.H = h;
    a.W = w;
    a.dk = dw_kernel;
    a.dy = dy;
    a.dz = dz;
    a.pw_slab = static_cast<float*>(ws);
    a.dw_slab = reinterpret_cast<float*>(static_cast<char*>(ws) + align_up((size_t)p.S * CI * CO * sizeof(float), 256));
    a.tiles = p.tiles;
    a.tps = p.tps;
    hipStream_t st = as_stream(stream);
    const bool drop = x->drop_rate > 0.f;
    switch (x->mode) {
        case UNET_VIEW_PLAIN:
            if (drop) launch_sw<UNET_VIEW_PLAIN, true>(a, p.S, st);
            else launch_sw<UNET_VIEW_PLAIN, false>(a, p.S, st);
            break;
        case UNET_VIEW_BNRELU:
            if (drop) launch_sw<UNET_VIEW_BNRELU, true>(a, p.S, st);
            else launch_sw<UNET_VIEW_BNRELU, false>(a, p.S, st);
            break;
        default:
            if (drop) launch_sw<UNET_VIEW_CONCAT, true>(a, p.S, st);
            else launch_sw<UNET_VIEW_CONCAT, false>(a, p.S, st);
            break;
    }
    UNET_CHECK_LAUNCH("unet_sepconv_bwd_filter");
    int rc = reduce_slabs(a.pw_slab, p.S, (int64_t)CI * CO, d_pw_kernel, (int64_t)CI * CO, (int64_t)CI * CO, st);
    if (rc) return rc;
    return reduce_slabs(a.dw_slab, p.S, (int64_t)9 * CI, d_dw_kernel, (int64_t)9 * CI, (int64_t)9 * CI, st);
}
