// Backward passes of a SeparableConv2D block that recompute the depthwise output y instead of
// reading it (reference model/u_net.py:14-25; the GradientTape of scripts/train.py:308):
//
//   d_pw[ci][co] = sum_px y[px][ci] dz[px][co]          y = depthwise3x3(x), recomputed here
//   d_dw[t][ci]  = sum_px x[px + off(t)][ci] dy[px][ci]  (the 3x3 taps y is formed from)
//
// x is the block's input VIEW (BN affine + ReLU / concat / dropout on load, zero padding).
//   * sepconv_bwd_fused_kernel (unet_sepconv_bwd_fused): the whole backward of a 64-output block
//     but its depthwise data gradient -- dz formed per tile from (da, z), dy = dz . pk^T, both
//     weight gradients; the train step's path for the 256 x 256 level (HBM-bound: the forward
//     keeps no y, dz never goes to memory);
//   * sepconv_bwd_filter2_kernel (unet_sepconv_bwd_filter): both weight gradients from dz and dy
//     in memory, 64 or 128 outputs.
// Both run 4-wave blocks over 4 x 16 pixel tiles, two blocks per CU; each block walks a run of
// tiles, one fixed-order slab per block, reduced by reduce_slabs in fixed order.
#include "common.h"
#include "view.h"

namespace unet {
namespace {

#ifndef SW_KO  // lab knock-outs (tools/lab/sw_fused_lab.hip): 1 weight-gradient MFMA, 2 depthwise VALU,
               // 4 loads of the next tile, 8 LDS staging, 16 the dy MFMA, 32 the dy store
#define SW_KO 0
#endif
constexpr int TH = 8, TW = 16;  // shape granularity of the C-ABI (h % 8, w % 16)
constexpr int CI = 64;          // input channels per block (ci group)
__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

struct SwArgs {
    DView x;
    int N, H, W, Cin;
    const float* dk;  // (3,3,Cin,1)
    const float* dy;  // (M, Cin)
    const float* dz;  // (M, CO)
    float* pw_slab;   // [S][Cin][CO]
    float* dw_slab;   // [S][9][Cin]
    int tiles, tps;   // pixel tiles, tiles per m-slice
    int ncig;         // ci groups of 64 channels
    // fused block backward (sepconv_bwd_fused_kernel: the whole backward of a 64-output conv block
    // but its depthwise data gradient): dz is formed per tile from the block's incoming gradient da
    // and raw z exactly as the BN-backward data-gradient GEMM forms it (gemm.hip A_BNBWD), dy =
    // dz . pk^T is computed there and written out (dy_out), and never goes through HBM as dz
    const float *da, *z, *coef, *bsc, *bsh, *pk;
    const float *da_dl, *da_k;  // rank-one da = da_dl[px] * da_k[c] (the binary head), da NULL
    float* dy_out;
};

// ------------------------------------------------------------------------------------------
// The fused block backward (unet_sepconv_bwd_fused): the whole backward of a 64-output conv block
// but its depthwise data gradient.  Per 4 x 16 pixel tile: dz formed from (da, z) into LDS, dy =
// dz . pk^T by MFMA (written out; dz never goes to HBM), y recomputed from the view's halo (the
// forward's fmaf chain) with the depthwise filter gradient from the same taps, then y^T dz by
// MFMA.  4-wave blocks, TWO per CU (77.5 KB of LDS each: the dy tile and the y tile share one
// buffer -- each thread reads its dy quad and writes its y quad at the same place).  The two resident blocks run their barrier-separated phases (staging, dy GEMM,
// depthwise, weight-gradient GEMM) independently, so one block's MFMAs overlap the other's
// loads, stores and VALU work; with one 8-wave block per CU every phase ran alone (lab knock-outs,
// tools/lab/sw_fused_lab.hip: each of the four phases cost 10-30 % of the kernel additively;
// this form: enc1_block2 320 -> 307 us, dec1_block1 597 -> 532 us, step +1.2 %).
// A block walks its run of tiles down a column (th fastest): consecutive tiles share two halo rows.
namespace fb {
constexpr int TH = 4, TW = 16, HWp = TW + 2, HPIX = (TH + 2) * HWp;  // 108 halo pixels
constexpr int PX = TH * TW;                                          // 64 pixels per tile
constexpr int NT = 256, CI = 64, CO = 64, ZS = CO + 1;
constexpr int NHQ = HPIX * (CI / 4);    // halo float4 (1728)
constexpr int HR = (NHQ + NT - 1) / NT;  // per thread (7)
constexpr int DQ = PX * (CO / 4) / NT;   // dz float4 per thread (4)
constexpr int L_X = HPIX * CI, L_YD = PX * CI, L_Z = PX * ZS, L_W = CO * CI, L_K = 9 * CI;
constexpr int SIZE = L_X + L_YD + L_Z + L_W + L_K;  // 19840 floats (77.5 KB)
static_assert(CI * CO <= SIZE && 9 * 16 * 16 * 4 <= SIZE, "epilogue scratch");
static_assert(2 * SIZE * 4 <= 160 * 1024, "two blocks per CU");
}  // namespace fb

template <int MODE, bool DA1 = false>
__global__ __launch_bounds__(fb::NT, 2) void sepconv_bwd_fused_kernel(SwArgs g) {
    constexpr int TH = fb::TH, TW = fb::TW, HWp = fb::HWp, PX = fb::PX, NT = fb::NT, CI = fb::CI, CO = fb::CO;
    constexpr int ZS = fb::ZS, NHQ = fb::NHQ, HR = fb::HR, DQ = fb::DQ;
    __shared__ __attribute__((aligned(16))) float smem[fb::SIZE];
    float* Xs = smem;
    float* YD = Xs + fb::L_X;  // dy tile [px][ci], then (in place) the y tile
    float* Zs = YD + fb::L_YD;
    float* Wt = Zs + fb::L_Z;  // [co][ci]
    float* KS9 = Wt + fb::L_W;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    const int j = blockIdx.x >> 3;  // XCD-aware (ci group, m-slice) map: the ci groups of a slice share an XCD
    // slices contiguous per XCD: XCD x runs slices [x S/8, (x+1) S/8), i.e. neighbouring tile columns,
    // so their shared halo columns meet in one L2 (S = gridDim.x / ncig, a multiple of 8)
    const int cig = j % g.ncig, slice = (int)(blockIdx.x & 7) * (int)(gridDim.x / g.ncig / 8) + j / g.ncig;
    const int c0 = CI * cig;
    const int t_begin = slice * g.tps;
    const int t_end = t_begin + g.tps < g.tiles ? t_begin + g.tps : g.tiles;
    const int tiles_h = g.H / TH;
    const int Cin = g.Cin;
    const int cq = tid & 15, ci = c0 + 4 * cq;

    for (int e = tid; e < 9 * CI; e += NT) KS9[e] = g.dk[(e / CI) * Cin + c0 + e % CI];
    for (int e = tid; e < CO * CI; e += NT) {  // Wt[co][ci] = pk[c0 + ci][co]
        const int co = e / CI, cl = e - co * CI;
        Wt[co * CI + cl] = g.pk[(int64_t)(c0 + cl) * CO + co];
    }
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
    // tile T: column-major walk (th fastest)
    auto tile_base = [&](int T, int& n, int& h0, int& w0) {
        const int th = T % tiles_h, r = T / tiles_h, tiles_w = g.W / TW;
        w0 = (r % tiles_w) * TW;
        n = r / tiles_w;
        h0 = th * TH;
    };
    float4 hx[HR], rz[DQ], rzz[DQ];
    bool hok[HR];
    auto load = [&](int T) {
        int n, h0, w0;
        tile_base(T, n, h0, w0);
#pragma unroll
        for (int k = 0; k < HR; ++k) {
            const int e = tid + NT * k;
            const int pix = e >> 4, r = pix / HWp, c = pix - r * HWp;
            const int hh = h0 - 1 + r, ww = w0 - 1 + c;
            hok[k] = e < NHQ && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
            hx[k] = ld4(src + ((int64_t)(hok[k] ? (n * g.H + hh) * g.W + ww : 0) * cs + cc));
        }
        const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
        for (int k = 0; k < DQ; ++k) {  // pixel (tid >> 4) + 16 k, output-channel quad cq
            const int p = (tid >> 4) + 16 * k;
            const int64_t px = mbase + (int64_t)(p >> 4) * g.W + (p & 15), o = px * CO + 4 * cq;
            if constexpr (DA1) rz[k].x = g.da_dl[px];  // (the 16 lanes of a pixel read one float)
            else rz[k] = ld4(g.da + o);
            rzz[k] = ld4(g.z + o);
        }
    };
    auto store = [&]() {
        // dz = sc (g - p - (z - mu) q), g = da [z sc + sh > 0] (as gemm.hip A_BNBWD); this thread's
        // output-channel quad is cq in every k (BN constants re-read: L1 hits)
        const float4 fsc = ld4(g.bsc + 4 * cq), fsh = ld4(g.bsh + 4 * cq);
        const float4 fmu = ld4(g.coef + 4 * cq), fp = ld4(g.coef + CO + 4 * cq), fq = ld4(g.coef + 2 * CO + 4 * cq);
        float4 fk = f4(0.f);
        if constexpr (DA1) fk = ld4(g.da_k + 4 * cq);
#pragma unroll
        for (int k = 0; k < HR; ++k) {
            const int e = tid + NT * k;
            float4 v = hx[k];
            if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (bn) v = bnrelu4(v, hsc, hsh);
            }
            if (!hok[k]) v = f4(0.f);
            if (e < NHQ) *reinterpret_cast<float4*>(&Xs[(e >> 4) * CI + 4 * (e & 15)]) = v;
        }
#pragma unroll
        for (int k = 0; k < DQ; ++k) {
            float4 v = rz[k];
            if constexpr (DA1) v = mul4(fk, f4(rz[k].x));  // the product unet_head_bwd would have stored
            const float4 zz = rzz[k];
            v.x = fmaf(zz.x, fsc.x, fsh.x) > 0.f ? v.x : 0.f;
            v.y = fmaf(zz.y, fsc.y, fsh.y) > 0.f ? v.y : 0.f;
            v.z = fmaf(zz.z, fsc.z, fsh.z) > 0.f ? v.z : 0.f;
            v.w = fmaf(zz.w, fsc.w, fsh.w) > 0.f ? v.w : 0.f;
            v.x = fsc.x * (v.x - fp.x - (zz.x - fmu.x) * fq.x);
            v.y = fsc.y * (v.y - fp.y - (zz.y - fmu.y) * fq.y);
            v.z = fsc.z * (v.z - fp.z - (zz.z - fmu.z) * fq.z);
            v.w = fsc.w * (v.w - fp.w - (zz.w - fmu.w) * fq.w);
            float* d = &Zs[((tid >> 4) + 16 * k) * ZS + 4 * cq];
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    };

    // dy GEMM: wave w -> pixels 32 (w >> 1) .., channels 32 (w & 1) ..; weight-gradient GEMM:
    // wave w -> the (32 ci x 32 co) quarter ci 32 (w & 1) .., co 32 (w >> 1) .. over all 64 pixels
    const int px0 = 32 * (wave >> 1), cl0 = 32 * (wave & 1);
    const int wci = 32 * (wave & 1), wco = 32 * (wave >> 1);
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float4 dwa[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) dwa[t] = f4(0.f);

    if (t_begin < t_end) load(t_begin);
    for (int T = t_begin; T < t_end; ++T) {
        if constexpr (!(SW_KO & 8)) store();
        __syncthreads();
        int n, h0, w0;
        tile_base(T, n, h0, w0);
        const int64_t tbase = (int64_t)(n * g.H + h0) * g.W + w0;
        if constexpr (!(SW_KO & 4)) load(T + 1 < t_end ? T + 1 : T);  // next tile in flight (past the end: a valid, unused tile)
        {
            floatx16 ad;
#pragma unroll
            for (int r = 0; r < 16; ++r) ad[r] = 0.f;
#pragma unroll 8
            for (int k = 0; k < ((SW_KO & 16) ? 0 : CO); k += 2)
                ad = __builtin_amdgcn_mfma_f32_32x32x2f32(Zs[(px0 + lo) * ZS + k + hi], Wt[(k + hi) * CI + cl0 + lo], ad,
                                                          0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) YD[(px0 + acc_row(r, hi)) * CI + cl0 + lo] = ad[r];
        }
        __syncthreads();
#pragma unroll 1
        for (int k = 0; k < ((SW_KO & 2) ? 0 : 4); ++k) {  // (not unrolled: 9 taps in flight, not 36)
            const int p = (tid >> 4) + 16 * k, pr = p >> 4, pc = p & 15;
            float4* yd = reinterpret_cast<float4*>(&YD[p * CI + 4 * cq]);
            const float4 dq = *yd;
            if constexpr (!(SW_KO & 32)) st4(g.dy_out + (tbase + (int64_t)pr * g.W + pc) * Cin + ci, dq);
            float4 y = f4(0.f);
#pragma unroll
            for (int dy_ = 0; dy_ < 3; ++dy_)
#pragma unroll
                for (int dx_ = 0; dx_ < 3; ++dx_) {
                    const float4 xv = *reinterpret_cast<const float4*>(&Xs[((pr + dy_) * HWp + pc + dx_) * CI + 4 * cq]);
                    y = fma4(xv, *reinterpret_cast<const float4*>(&KS9[(dy_ * 3 + dx_) * CI + 4 * cq]), y);
                    dwa[dy_ * 3 + dx_] = fma4(xv, dq, dwa[dy_ * 3 + dx_]);
                }
            *yd = y;  // the same thread read this slot's dy above
        }
        __syncthreads();
#pragma unroll 4
        for (int s = 0; s < ((SW_KO & 1) ? 0 : PX / 2); ++s) {
            const int p = 2 * s + hi;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(YD[p * CI + wci + lo], Zs[p * ZS + wco + lo], acc, 0, 0, 0);
        }
        __syncthreads();
    }

    float* E = smem;  // pointwise slab rows c0 .. c0+63: [64 ci][CO]
#pragma unroll
    for (int r = 0; r < 16; ++r) E[(wci + acc_row(r, hi)) * CO + wco + lo] = acc[r];
    __syncthreads();
    float* pw = g.pw_slab + ((int64_t)slice * Cin + c0) * CO;
    for (int e = tid; e < CI * CO / 4; e += NT) st4(pw + 4 * e, *reinterpret_cast<const float4*>(&E[4 * e]));
    __syncthreads();
    // depthwise slab [t][ci]: the 16 threads of each channel quad, fixed-order tree
    float4* D = reinterpret_cast<float4*>(smem);  // [9][16 pixel rows][16 quads]
#pragma unroll
    for (int t = 0; t < 9; ++t) D[(t * 16 + (tid >> 4)) * 16 + cq] = dwa[t];
    __syncthreads();
    for (int o = 8; o > 0; o >>= 1) {
        for (int e = tid; e < 9 * o * 16; e += NT) {
            const int t = e / (o * 16), rr = (e / 16) % o, q = e % 16;
            D[(t * 16 + rr) * 16 + q] = add4(D[(t * 16 + rr) * 16 + q], D[(t * 16 + rr + o) * 16 + q]);
        }
        __syncthreads();
    }
    float* dws = g.dw_slab + (int64_t)slice * 9 * Cin;
    if (tid < 9 * 16) st4(dws + (tid / 16) * Cin + c0 + 4 * (tid % 16), D[(tid / 16) * 16 * 16 + (tid % 16)]);
}

// Both weight gradients WITHOUT the data path (unet_sepconv_bwd_filter: dz and dy come from
// memory), in the fused kernel's form: 4-wave blocks over 4 x 16 pixel tiles, two per CU, 64 or 128
// outputs, dropout on the view.  Per tile: the view's halo and the dz tile -> LDS, y recomputed
// with the forward's fmaf chain (taps from LDS) while the depthwise-filter gradient accumulates
// against this thread's dy quads, then y^T dz by MFMA (wave w: ci 32 (w & 1) .., co quarters
// 32 (CO/64 (w >> 1) + q) ..).  The next tile's halo / dz loads and dy quads are in flight meanwhile.
template <int CO>
struct Fw2Lds {
    static constexpr int SIZE = fb::L_X + fb::L_YD + fb::PX * CO + fb::L_K;  // 77.3 KB (CO 128) / 61 KB (CO 64)
    static_assert(fb::CI * CO <= SIZE && 9 * 16 * 16 * 4 <= SIZE, "epilogue scratch");
    static_assert(2 * SIZE * 4 <= 160 * 1024, "two blocks per CU");
};

template <int MODE, bool DROP, int CO>
__global__ __launch_bounds__(fb::NT, 2) void sepconv_bwd_filter2_kernel(SwArgs g) {
    constexpr int TH = fb::TH, TW = fb::TW, HWp = fb::HWp, PX = fb::PX, NT = fb::NT, CI = fb::CI;
    constexpr int NHQ = fb::NHQ, HR = fb::HR;
    constexpr int DQ = PX * (CO / 4) / NT;  // dz float4 per thread per tile (4 / 8)
    constexpr int NQW = CO / 64;            // (32 ci x 32 co) quarters per wave
    __shared__ __attribute__((aligned(16))) float smem[Fw2Lds<CO>::SIZE];
    float* Xs = smem;
    float* Ys = Xs + fb::L_X;
    float* Zs = Ys + fb::L_YD;
    float* KS9 = Zs + PX * CO;  // the ci group's 9 taps [t][ci] (in LDS: registers go to the dz staging)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    const int j = blockIdx.x >> 3;  // XCD-aware (ci group, m-slice) map, as the fused kernel
    // slices contiguous per XCD: XCD x runs slices [x S/8, (x+1) S/8), i.e. neighbouring tile columns,
    // so their shared halo columns meet in one L2 (S = gridDim.x / ncig, a multiple of 8)
    const int cig = j % g.ncig, slice = (int)(blockIdx.x & 7) * (int)(gridDim.x / g.ncig / 8) + j / g.ncig;
    const int c0 = CI * cig;
    const int t_begin = slice * g.tps;
    const int t_end = t_begin + g.tps < g.tiles ? t_begin + g.tps : g.tiles;
    const int tiles_h = g.H / TH;
    const int C = g.x.C, Cin = g.Cin;
    const int cq = tid & 15, ci = c0 + 4 * cq;

    for (int e = tid; e < 9 * CI; e += NT) KS9[e] = g.dk[(e / CI) * Cin + c0 + e % CI];
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
    auto tile_base = [&](int T) {  // first pixel of tile T (column-major walk, th fastest)
        const int th = T % tiles_h, r = T / tiles_h, tiles_w = g.W / TW;
        return (int64_t)((r / tiles_w) * g.H + th * TH) * g.W + (r % tiles_w) * TW;
    };
    float4 hx[HR], rz[DQ], rdy[4];
    // halo element k of this thread in tile T: its pixel index, or -1 outside the image (recomputed
    // where needed instead of held in registers across the tile)
    auto halo_px = [&](int T, int k) {
        const int th = T % tiles_h, r = T / tiles_h, tiles_w = g.W / TW;
        const int n = r / tiles_w, h0 = th * TH, w0 = (r % tiles_w) * TW;
        const int e = tid + NT * k;
        const int pix = e >> 4, rr = pix / HWp, c = pix - rr * HWp;
        const int hh = h0 - 1 + rr, ww = w0 - 1 + c;
        const bool ok = e < NHQ && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
        return ok ? (n * g.H + hh) * g.W + ww : -1;
    };
    auto load = [&](int T) {
        const int th = T % tiles_h, r = T / tiles_h, tiles_w = g.W / TW;
        const int n = r / tiles_w, h0 = th * TH, w0 = (r % tiles_w) * TW;
#pragma unroll
        for (int k = 0; k < HR; ++k) {
            const int lp = halo_px(T, k);
            hx[k] = ld4(src + ((int64_t)(lp < 0 ? 0 : lp) * cs + cc));
        }
        const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
        for (int k = 0; k < DQ; ++k) {  // dz tile: element e = pixel e / (CO/4), quad e % (CO/4)
            const int e = tid + NT * k, p = e / (CO / 4), q = e % (CO / 4);
            rz[k] = ld4(g.dz + (mbase + (int64_t)(p >> 4) * g.W + (p & 15)) * CO + 4 * q);
        }
    };
    auto load_dy = [&](int T) {  // this thread's dy quads: pixel (tid >> 4) + 16 k
        const int64_t tb = tile_base(T);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = (tid >> 4) + 16 * k;
            rdy[k] = ld4(g.dy + (tb + (int64_t)(p >> 4) * g.W + (p & 15)) * Cin + ci);
        }
    };
    auto store = [&](int T) {
#pragma unroll
        for (int k = 0; k < HR; ++k) {
            const int e = tid + NT * k;
            const int lp = halo_px(T, k);
            float4 v = hx[k];
            if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (bn) v = bnrelu4(v, hsc, hsh);
            }
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)(lp < 0 ? 0 : lp) * C + ci;
                v = mul4(v, drop_mult4(g.x.seed, i, g.x.rate, g.x.inv_keep));
            }
            if (lp < 0) v = f4(0.f);
            if (e < NHQ) *reinterpret_cast<float4*>(&Xs[(e >> 4) * CI + 4 * (e & 15)]) = v;
        }
#pragma unroll
        for (int k = 0; k < DQ; ++k) {
            const int e = tid + NT * k;
            *reinterpret_cast<float4*>(&Zs[(e / (CO / 4)) * CO + 4 * (e % (CO / 4))]) = rz[k];
        }
    };

    const int wci = 32 * (wave & 1), wco = 32 * NQW * (wave >> 1);
    floatx16 acc[NQW];
#pragma unroll
    for (int q = 0; q < NQW; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
    float4 dwa[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) dwa[t] = f4(0.f);

    if (t_begin < t_end) {
        load(t_begin);
        load_dy(t_begin);
    }
    for (int T = t_begin; T < t_end; ++T) {
        store(T);
        __syncthreads();
        load(T + 1 < t_end ? T + 1 : T);  // next tile in flight (past the end: a valid, unused tile)
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {  // (not unrolled: 9 taps in flight, not 36)
            const int p = (tid >> 4) + 16 * k, pr = p >> 4, pc = p & 15;
            const float4 dq = rdy[0];  // static register indexing: rotate the dy quads
            rdy[0] = rdy[1];
            rdy[1] = rdy[2];
            rdy[2] = rdy[3];
            float4 y = f4(0.f);
#pragma unroll
            for (int dy_ = 0; dy_ < 3; ++dy_)
#pragma unroll
                for (int dx_ = 0; dx_ < 3; ++dx_) {
                    const float4 xv = *reinterpret_cast<const float4*>(&Xs[((pr + dy_) * HWp + pc + dx_) * CI + 4 * cq]);
                    y = fma4(xv, *reinterpret_cast<const float4*>(&KS9[(dy_ * 3 + dx_) * CI + 4 * cq]), y);
                    dwa[dy_ * 3 + dx_] = fma4(xv, dq, dwa[dy_ * 3 + dx_]);
                }
            *reinterpret_cast<float4*>(&Ys[p * CI + 4 * cq]) = y;
        }
        load_dy(T + 1 < t_end ? T + 1 : T);  // its latency hides behind the MFMA phase
        __syncthreads();
#pragma unroll 4
        for (int s2 = 0; s2 < PX / 2; ++s2) {
            const int p = 2 * s2 + hi;
            const float a = Ys[p * CI + wci + lo];
#pragma unroll
            for (int q = 0; q < NQW; ++q)
                acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Zs[p * CO + wco + 32 * q + lo], acc[q], 0, 0, 0);
        }
        __syncthreads();
    }

    float* E = smem;  // pointwise slab rows c0 .. c0+63: [64 ci][CO]
#pragma unroll
    for (int q = 0; q < NQW; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) E[(wci + acc_row(r, hi)) * CO + wco + 32 * q + lo] = acc[q][r];
    __syncthreads();
    float* pw = g.pw_slab + ((int64_t)slice * Cin + c0) * CO;
    for (int e = tid; e < CI * CO / 4; e += NT) st4(pw + 4 * e, *reinterpret_cast<const float4*>(&E[4 * e]));
    __syncthreads();
    float4* D = reinterpret_cast<float4*>(smem);  // [9][16 pixel rows][16 quads]
#pragma unroll
    for (int t = 0; t < 9; ++t) D[(t * 16 + (tid >> 4)) * 16 + cq] = dwa[t];
    __syncthreads();
    for (int o = 8; o > 0; o >>= 1) {
        for (int e = tid; e < 9 * o * 16; e += NT) {
            const int t = e / (o * 16), rr = (e / 16) % o, q = e % 16;
            D[(t * 16 + rr) * 16 + q] = add4(D[(t * 16 + rr) * 16 + q], D[(t * 16 + rr + o) * 16 + q]);
        }
        __syncthreads();
    }
    float* dws = g.dw_slab + (int64_t)slice * 9 * Cin;
    if (tid < 9 * 16) st4(dws + (tid / 16) * Cin + c0 + 4 * (tid % 16), D[(tid / 16) * 16 * 16 + (tid % 16)]);
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
    int tiles, ncig, S, tps;
};
SwPlan sw_plan(int n, int h, int w, int cin) {
    SwPlan p;
    p.tiles = n * (h / fb::TH) * (w / fb::TW);
    p.ncig = cin / CI;
    // two blocks per CU (77 KB of LDS each), m-slices a multiple of 8 (the XCD map).  (Fewer blocks,
    // leaving CUs to the main stream: -1.7 / -0.3 % img/s in round 2; 2-8x as many, finer runs:
    // no gain, profiles/r3m_fb_split_ab.log.)
    int S = (int)cdiv(2 * resident_cus(), p.ncig);
    S = (int)cdiv(S, 8) * 8;
    p.tps = (int)cdiv(p.tiles, S);
    p.S = S;
    return p;
}

template <int MODE, bool DROP>
void launch_sw(const SwArgs& a, int cout, int blocks, hipStream_t st) {
    if (a.da_dl) sepconv_bwd_fused_kernel<MODE, true><<<blocks, fb::NT, 0, st>>>(a);
    else if (a.da) sepconv_bwd_fused_kernel<MODE><<<blocks, fb::NT, 0, st>>>(a);
    else if (cout == 128) sepconv_bwd_filter2_kernel<MODE, DROP, 128><<<blocks, fb::NT, 0, st>>>(a);
    else sepconv_bwd_filter2_kernel<MODE, DROP, 64><<<blocks, fb::NT, 0, st>>>(a);
}

}  // namespace
}  // namespace unet

using namespace unet;

extern "C" int unet_sepconv_bwd_filter_supported(const unet_view* x, int n, int h, int w, int cout) {
    // 64 outputs (the 256 x 256 level) or 128 (the 128 x 128 level: 142 KB of LDS; isolated it is
    // slower than the separate launches, 224 vs 188 us in tools/bench_sepwgrad.py, but it lets the
    // forward skip the y store -- the engine chooses per level)
    if (!x || n <= 0 || h <= 0 || w <= 0 || (cout != 64 && cout != 128)) return 0;
    if (x->mode != UNET_VIEW_PLAIN && x->mode != UNET_VIEW_BNRELU && x->mode != UNET_VIEW_CONCAT) return 0;
    const int C = x->c0 + (x->mode == UNET_VIEW_CONCAT ? x->c1 : 0);
    if (C % CI || h % TH || w % TW) return 0;
    if (x->mode == UNET_VIEW_CONCAT && x->c0 % 4) return 0;
    const int64_t M = (int64_t)n * h * w;
    return M * C < (int64_t(1) << 31) && M * cout < (int64_t(1) << 31);
}

extern "C" size_t unet_sepconv_bwd_filter_workspace(int n, int h, int w, int cin, int cout) {
    if (n <= 0 || h <= 0 || w <= 0 || cin <= 0 || cin % CI || (cout != 64 && cout != 128) || h % TH || w % TW)
        return 0;
    const SwPlan p = sw_plan(n, h, w, cin);
    return align_up((size_t)p.S * cin * cout * sizeof(float), 256) + align_up((size_t)p.S * 9 * cin * sizeof(float), 256);
}

namespace {
int run_sw(const unet_view* x, int n, int h, int w, const float* dw_kernel, SwArgs a, int cout, float* d_dw_kernel,
           float* d_pw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream, const char* op) {
    const int cin = x->c0 + (x->mode == UNET_VIEW_CONCAT ? x->c1 : 0);
    const size_t need = unet_sepconv_bwd_filter_workspace(n, h, w, cin, cout);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "%s: workspace %zu < %zu", op, ws_bytes, need);
    const SwPlan p = sw_plan(n, h, w, cin);
    a.x = make_dview(*x);
    a.N = n;
    a.H = h;
    a.W = w;
    a.Cin = cin;
    a.dk = dw_kernel;
    a.pw_slab = static_cast<float*>(ws);
    a.dw_slab = reinterpret_cast<float*>(static_cast<char*>(ws) + align_up((size_t)p.S * cin * cout * sizeof(float), 256));
    a.tiles = p.tiles;
    a.tps = p.tps;
    a.ncig = p.ncig;
    const int blocks = p.S * p.ncig;
    hipStream_t st = as_stream(stream);
    const bool drop = x->drop_rate > 0.f;
    switch (x->mode) {
        case UNET_VIEW_PLAIN:
            if (drop) launch_sw<UNET_VIEW_PLAIN, true>(a, cout, blocks, st);
            else launch_sw<UNET_VIEW_PLAIN, false>(a, cout, blocks, st);
            break;
        case UNET_VIEW_BNRELU:
            if (drop) launch_sw<UNET_VIEW_BNRELU, true>(a, cout, blocks, st);
            else launch_sw<UNET_VIEW_BNRELU, false>(a, cout, blocks, st);
            break;
        default:
            if (drop) launch_sw<UNET_VIEW_CONCAT, true>(a, cout, blocks, st);
            else launch_sw<UNET_VIEW_CONCAT, false>(a, cout, blocks, st);
            break;
    }
    UNET_CHECK_LAUNCH(op);
    const int64_t lp = (int64_t)cin * cout, ld = (int64_t)9 * cin;
    return reduce_slabs_pair(a.pw_slab, lp, d_pw_kernel, a.dw_slab, ld, d_dw_kernel, p.S, st);
}
}  // namespace

extern "C" int unet_sepconv_bwd_fused(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                                      const float* pw_kernel, const float* da, const float* da_dlogit,
                                      const float* da_kernel, const float* z, const float* scale,
                                      const float* shift, const float* coef, int cout, float* dy, float* d_dw_kernel,
                                      float* d_pw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream) {
    const char* op = "unet_sepconv_bwd_fused";
    if (check_view(x, op)) return -1;
    UNET_CHECK_ARG(cout == 64 && unet_sepconv_bwd_filter_supported(x, n, h, w, cout) && x->drop_rate == 0.f,
                   "%s: unsupported (needs 64 output channels, input channels %% 64 == 0, no dropout on the input, "
                   "a PLAIN / BNRELU / CONCAT view, h %% 8 == 0, w %% 16 == 0)", op);
    UNET_CHECK_ARG(dw_kernel && pw_kernel && z && scale && shift && coef && dy && d_dw_kernel && d_pw_kernel,
                   "%s: null pointer", op);
    UNET_CHECK_ARG(da ? !da_dlogit && !da_kernel : da_dlogit && da_kernel,
                   "%s: give da, or da_dlogit and da_kernel (rank-one da)", op);
    UNET_CHECK_ARG(((uintptr_t)da | (uintptr_t)da_kernel | (uintptr_t)z | (uintptr_t)dy | (uintptr_t)scale | (uintptr_t)shift |
                    (uintptr_t)coef | (uintptr_t)dw_kernel | (uintptr_t)x->src0 |
                    (uintptr_t)(x->src1 ? x->src1 : x->src0)) % 16 == 0,
                   "%s: operands must be 16-B aligned", op);
    SwArgs a{};
    a.da = da;
    a.da_dl = da_dlogit;
    a.da_k = da_kernel;
    a.z = z;
    a.coef = coef;
    a.bsc = scale;
    a.bsh = shift;
    a.pk = pw_kernel;
    a.dy_out = dy;
    return run_sw(x, n, h, w, dw_kernel, a, cout, d_dw_kernel, d_pw_kernel, ws, ws_bytes, stream, op);
}

extern "C" int unet_sepconv_bwd_filter(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                                       const float* dy, const float* dz, int cout, float* d_dw_kernel,
                                       float* d_pw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream) {
    if (check_view(x, "unet_sepconv_bwd_filter")) return -1;
    UNET_CHECK_ARG(unet_sepconv_bwd_filter_supported(x, n, h, w, cout),
                   "unet_sepconv_bwd_filter: unsupported shape (needs input channels %% 64 == 0, 64 or 128 "
                   "output channels, a PLAIN / BNRELU / CONCAT view, h %% 8 == 0, w %% 16 == 0)");
    UNET_CHECK_ARG(dw_kernel && dy && dz && d_dw_kernel && d_pw_kernel, "unet_sepconv_bwd_filter: null pointer");
    UNET_CHECK_ARG(((uintptr_t)dy | (uintptr_t)dz | (uintptr_t)dw_kernel | (uintptr_t)x->src0 |
                    (uintptr_t)(x->src1 ? x->src1 : x->src0)) % 16 == 0,
                   "unet_sepconv_bwd_filter: operands must be 16-B aligned");
    SwArgs a{};
    a.dy = dy;
    a.dz = dz;
    return run_sw(x, n, h, w, dw_kernel, a, cout, d_dw_kernel, d_pw_kernel, ws, ws_bytes, stream,
                  "unet_sepconv_bwd_filter");
}
