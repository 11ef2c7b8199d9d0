// Tiled depthwise 3x3 kernels (the fast path of unet_dwconv3x3_*; reference op:
// DepthwiseConv2dNative of SeparableConv2D, model/u_net.py:14-20).
//
// A block owns an 8 x TW pixel tile of one image and a chunk of 4*QT channels (TW = 256/QT,
// so every lane owns one tile column x one channel quad).  The (8+2) x (TW+2) halo of the
// input is staged into LDS ONCE, through the activation view (BN affine + ReLU, 2x2 max-pool,
// concat, dropout are applied once per staged element instead of once per tap), then each
// lane walks its column with a rolling 3-row register window: 3 ds_read_b128 per output
// quad instead of 9.  HBM traffic ~ input x (1 + halo overhead) + output; the halo re-reads of
// neighbouring tiles hit L2.  The weight gradient uses the same staging and accumulates the 9
// tap sums in registers over a persistent loop of tiles, then one fixed-order LDS reduction
// per block -> deterministic per-block partials.
#include "view.h"

namespace unet {

int dw_tiled_fwd(const DView& v, int mode, bool drop, int N, int H, int W, const float* K, float* Y, hipStream_t st);
int dw_tiled_bwd_data(const DView& v, int mode, bool drop, int N, int H, int W, const float* K, const float* dY,
                      float* dx0, float* dx1, hipStream_t st);
size_t dw_tiled_filter_partials(int N, int H, int W, int C);
int dw_tiled_bwd_data_bnstats(const DView& v, int mode, bool drop, int N, int H, int W, const float* K,
                              const float* dY, float* dx0, const float* mu, const float* rs, float* bnpart,
                              hipStream_t st, float* dwpart = nullptr);
size_t dw_tiled_ntiles(int N, int H, int W, int C);
int dw_tiled_bwd_filter(const DView& v, int mode, bool drop, int N, int H, int W, const float* dY, float* part,
                        int* S_out, hipStream_t st);
bool dw_tiled_ok(int C);

namespace {

constexpr int TH = 8;

template <int QT>
struct Geom {
    static constexpr int TW = 256 / QT;
    static constexpr int HWp = TW + 2;
    static constexpr int HHp = TH + 2;
    static constexpr int NE = HHp * HWp * QT;
};

// halo tile rows h0-1..h0+TH, cols w0-1..w0+TW, channels [cbase, cbase + 4 QT), zero outside.
// All loads of the tile are issued first (clamped, branch-free addresses), then transformed and
// stored, so the compiler does not wait on each load before issuing the next.
template <int MODE, bool DROP, int QT, int KBMAX = 1 << 20>
__device__ __forceinline__ void stage(float4* T, const DView& v, int n, int h0, int w0, int H, int W, int cbase) {
    using G = Geom<QT>;
    constexpr int NR = (G::NE + 255) / 256;
    constexpr int NP = MODE == UNET_VIEW_POOL_BNRELU ? 4 : 1;
    const int q = threadIdx.x % QT;  // 256 % QT == 0: the channel quad is fixed per thread
    const int c = cbase + 4 * q;
    // CONCAT: [raw upsample | bnrelu(skip)]; the selection is by value (no indexing into v)
    const bool second = MODE == UNET_VIEW_CONCAT && c >= v.c0;
    const float* src = second ? v.src1 : v.src0;
    const int cs = second ? v.c1 : v.c0;
    const int ci = second ? c - v.c0 : c;
    const bool bn = MODE == UNET_VIEW_BNRELU || MODE == UNET_VIEW_POOL_BNRELU || second;
    const float* scp = second ? v.sc1 : v.sc0;
    const float* shp = second ? v.sh1 : v.sh0;
    float4 sc = f4(1.f), sh = f4(0.f);
    if constexpr (MODE != UNET_VIEW_PLAIN) {
        if (bn) {
            sc = ld4(scp + ci);
            sh = ld4(shp + ci);
        }
    }
    // Loads of a batch of KB elements are issued back to back, then each element is transformed,
    // masked and written to LDS.  Non-pool views take the whole tile as one batch; the pool view
    // reads 4 sources per element and uses batches of 3 (12 loads in flight) to bound registers.
    constexpr int KB0 = NP == 4 ? 3 : NR;
    constexpr int KB = KB0 < KBMAX ? KB0 : KBMAX;
#pragma unroll
    for (int k0 = 0; k0 < NR; k0 += KB) {
        float4 pr[KB][NP];
        int lp[KB];
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
            const int e = threadIdx.x + 256 * (k0 + kk);
            const int pix = e / QT;
            const int r = pix / G::HWp;
            const int cc = pix - r * G::HWp;
            const int hh = h0 - 1 + r, ww = w0 - 1 + cc;
            const bool ok = k0 + kk < NR && e < G::NE && hh >= 0 && hh < H && ww >= 0 && ww < W;
            lp[kk] = ok ? (n * H + hh) * W + ww : -1;
            int sp = 0;
            if (ok) {
                if constexpr (MODE == UNET_VIEW_POOL_BNRELU) sp = (n * 2 * H + 2 * hh) * (2 * W) + 2 * ww;
                else sp = lp[kk];
            }
            const float* b = src + ((int64_t)sp * cs + ci);
            pr[kk][0] = ld4(b);
            if constexpr (NP == 4) {
                const int64_t rs = (int64_t)2 * W * cs;
                pr[kk][1] = ld4(b + cs);
                pr[kk][2] = ld4(b + rs);
                pr[kk][3] = ld4(b + rs + cs);
            }
        }
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
            const int e = threadIdx.x + 256 * (k0 + kk);
            float4 val = pr[kk][0];
            if constexpr (NP == 4) {
                val = fma4(val, sc, sh);
                val = max4(val, fma4(pr[kk][1], sc, sh));
                val = max4(val, fma4(pr[kk][2], sc, sh));
                val = max4(val, fma4(pr[kk][3], sc, sh));
                val = relu4(val);
            } else if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (bn) val = bnrelu4(val, sc, sh);
            }
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)(lp[kk] < 0 ? 0 : lp[kk]) * v.C + c;
                val = mul4(val, drop_mult4(v.seed, i, v.rate, v.inv_keep));
            }
            if (lp[kk] < 0) val = f4(0.f);
            if (k0 + kk < NR && e < G::NE) T[e] = val;
        }
    }
}

// XCD-aware tile order: workgroups go to the 8 XCDs round-robin by linear id, so neighbouring tiles
// (which re-read each other's halo rows and columns) would each run on a different XCD, i.e. behind a
// different L2.  With the tile count a multiple of 8, XCD x instead takes the contiguous run of tiles
// [x T/8, (x+1) T/8) in order: a tile's neighbours are resident on the same XCD and its halo reads
// hit that L2.  Same tiles, same arithmetic, same per-tile slabs -- only the placement changes.
__device__ __forceinline__ int xcd_tile(int b, int tiles) {
    return (tiles & 7) == 0 ? (b & 7) * (tiles >> 3) + (b >> 3) : b;
}

__device__ __forceinline__ void tile_coords(int b, int tiles_w, int tiles_h, int TW, int& n, int& h0, int& w0) {
    const int tw = b % tiles_w;
    b /= tiles_w;
    const int th = b % tiles_h;
    n = b / tiles_h;
    h0 = th * TH;
    w0 = tw * TW;
}

template <int MODE, bool DROP, int QT>
__global__ __launch_bounds__(256, 3) void dw_tile_fwd(DView v, int N, int H, int W, int tiles_w, int tiles_h,
                                                   const float* __restrict__ K, float* __restrict__ Y) {
    using G = Geom<QT>;
    __shared__ float4 T[G::NE];
    int n, h0, w0;
    tile_coords(xcd_tile(blockIdx.x, gridDim.x), tiles_w, tiles_h, G::TW, n, h0, w0);
    const int cbase = blockIdx.y * 4 * QT;
    stage<MODE, DROP, QT>(T, v, n, h0, w0, H, W, cbase);
    const int q = threadIdx.x % QT, col = threadIdx.x / QT;
    const int C = v.C, c = cbase + 4 * q;
    float4 k[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) k[t] = ld4(K + t * C + c);
    __syncthreads();
    const int w = w0 + col;
    float4 a[3][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) a[i][j] = T[(i * G::HWp + col + j) * QT + q];
#pragma unroll
    for (int r = 0; r < TH; ++r) {
#pragma unroll
        for (int j = 0; j < 3; ++j) a[2][j] = T[((r + 2) * G::HWp + col + j) * QT + q];
        float4 acc = f4(0.f);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) acc = fma4(a[i][j], k[i * 3 + j], acc);
        if (w < W && h0 + r < H) st4(Y + ((int64_t)(n * H + h0 + r) * W + w) * C + c, acc);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            a[0][j] = a[1][j];
            a[1][j] = a[2][j];
        }
    }
}

// DWF (BNRELU view with STATS, no dropout): the depthwise FILTER gradient of the same layer from the
// same registers: dK[t][c] = sum_p x[p + off(t)] dy[p] = sum_q x[q] dy[q - off(t)] (both zero outside
// the image), and for the lane's output pixel q the staged dy window holds dy[q - off(t)] at
// a[2 - i][2 - j] (t = 3 i + j) while x[q] = relu(z sc + sh) comes from the z the statistics read
// anyway: 9 FMAs per element on the HBM-bound pass instead of a second pass over dy and the view
// (round 6).  Per tile a fixed-order [9][C] slab (xor shuffles over the wave's columns, then the
// four waves in order) into dwpart[tile]; unet_reduce_slabs sums the tiles in order.
// STATS (POOL or BNRELU view): this kernel is the last writer of the view's block's da (POOL: it
// adds the pooled half to the stored skip half and reads the block's raw z for the argmax anyway;
// BNRELU: it writes the whole da and reads z for the mask), so it also emits that block's
// BatchNorm-backward partial sums over its tile: bnpart[tile][0][c] = sum g,
// bnpart[tile][1][c] = sum g * xhat with g = da * [z*sc+sh > 0], xhat = (z - mu) * rs (the
// unet_bn_relu_bwd_stats reduction, without its separate pass over (da, z)).
template <int MODE, bool DROP, int QT, bool STATS = false, bool DWF = false>
__global__ __launch_bounds__(256, DWF ? 2 : 3) void dw_tile_bwd_data(DView v, int N, int H, int W, int tiles_w, int tiles_h,
                                                        const float* __restrict__ K, const float* __restrict__ dY,
                                                        float* __restrict__ dx0, float* __restrict__ dx1,
                                                        const float* __restrict__ mu = nullptr,
                                                        const float* __restrict__ rs = nullptr,
                                                        float* __restrict__ bnpart = nullptr,
                                                        float* __restrict__ dwpart = nullptr) {
    static_assert(!DWF || (STATS && MODE == UNET_VIEW_BNRELU && !DROP), "DWF: BNRELU view, statistics, no dropout");
    main_stream_prio();
    using G = Geom<QT>;
    __shared__ float4 T[G::NE];
    int n, h0, w0;
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    tile_coords(tile, tiles_w, tiles_h, G::TW, n, h0, w0);
    const int cbase = blockIdx.y * 4 * QT;
    const int C = v.C;
    DView dv{};
    dv.src0 = dY;
    dv.c0 = C;
    dv.C = C;
    stage<UNET_VIEW_PLAIN, false, QT>(T, dv, n, h0, w0, H, W, cbase);
    const int q = threadIdx.x % QT, col = threadIdx.x / QT;
    const int c = cbase + 4 * q;
    float4 kf[9];  // flipped kernel: dx(h,w) = sum dy(h-i+1, w-j+1) k[i][j]
#pragma unroll
    for (int t = 0; t < 9; ++t) kf[t] = ld4(K + (8 - t) * C + c);
    __syncthreads();
    const int w = w0 + col;
    float4 s1 = f4(0.f), s2 = f4(0.f);  // STATS partial sums of this thread's pixels
    float4 smu = f4(0.f), srs = f4(0.f);
    if constexpr (STATS) {
        if (mu) {
            smu = ld4(mu + c);
            srs = ld4(rs + c);
        }
    }
    float4 a[3][3];
    float4 fk[DWF ? 9 : 1];  // DWF: this lane's filter-gradient sums
    float4 xsc = f4(1.f), xsh = f4(0.f);
    if constexpr (DWF) {
#pragma unroll
        for (int t = 0; t < 9; ++t) fk[t] = f4(0.f);
        xsc = ld4(v.sc0 + c);
        xsh = ld4(v.sh0 + c);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) a[i][j] = T[(i * G::HWp + col + j) * QT + q];
#pragma unroll
    for (int r = 0; r < TH; ++r) {
#pragma unroll
        for (int j = 0; j < 3; ++j) a[2][j] = T[((r + 2) * G::HWp + col + j) * QT + q];
        float4 acc = f4(0.f);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) acc = fma4(a[i][j], kf[i * 3 + j], acc);
        float4 zq = f4(0.f);
        if constexpr (DWF) {  // x[q] (zero past the image) against the window's dy[q - off(t)]
            const bool in = w < W && h0 + r < H;
            zq = ld4(v.src0 + (in ? ((int64_t)(n * H + h0 + r) * W + w) * C + c : 0));
            float4 xq = bnrelu4(zq, xsc, xsh);
            if (!in) xq = f4(0.f);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) fk[i * 3 + j] = fma4(xq, a[2 - i][2 - j], fk[i * 3 + j]);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            a[0][j] = a[1][j];
            a[1][j] = a[2][j];
        }
        const int h = h0 + r;
        if (w >= W || h >= H) continue;
        const int p = (n * H + h) * W + w;
        if constexpr (DROP) {
            const uint64_t li = (uint64_t)p * C + c;
            acc = mul4(acc, drop_mult4(v.seed, li, v.rate, v.inv_keep));
        }
        if constexpr (MODE == UNET_VIEW_PLAIN || MODE == UNET_VIEW_BNRELU) {
            st4(dx0 + (int64_t)p * C + c, acc);
            if constexpr (STATS && MODE == UNET_VIEW_BNRELU) {  // dx0 is the whole da of the view's block
                const float4 zr = DWF ? zq : ld4(v.src0 + (int64_t)p * C + c);
                const float4 sc = ld4(v.sc0 + c), sh = ld4(v.sh0 + c);
                const float4 gm = make_float4(fmaf(zr.x, sc.x, sh.x) > 0.f ? acc.x : 0.f,
                                              fmaf(zr.y, sc.y, sh.y) > 0.f ? acc.y : 0.f,
                                              fmaf(zr.z, sc.z, sh.z) > 0.f ? acc.z : 0.f,
                                              fmaf(zr.w, sc.w, sh.w) > 0.f ? acc.w : 0.f);
                s1 = add4(s1, gm);
                const float4 xh = make_float4((zr.x - smu.x) * srs.x, (zr.y - smu.y) * srs.y,
                                              (zr.z - smu.z) * srs.z, (zr.w - smu.w) * srs.w);
                s2 = fma4(gm, xh, s2);
            }
        } else if constexpr (MODE == UNET_VIEW_CONCAT) {
            if (c < v.c0)
                st4(dx0 + (int64_t)p * v.c0 + c, acc);
            else
                st4(dx1 + (int64_t)p * v.c1 + (c - v.c0), acc);
        } else {  // POOL_BNRELU: gradient to the first max of the 2x2 window, accumulated
            const int W2 = 2 * W;
            const int64_t b = ((int64_t)(n * 2 * H + 2 * h) * W2 + 2 * w) * v.c0 + c;
            const int64_t off[4] = {0, v.c0, (int64_t)W2 * v.c0, (int64_t)W2 * v.c0 + v.c0};
            const float4 sc = ld4(v.sc0 + c), sh = ld4(v.sh0 + c);
            float4 zr[4], xv[4], g[4];
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                zr[qq] = ld4(v.src0 + b + off[qq]);
                xv[qq] = bnrelu4(zr[qq], sc, sh);
                g[qq] = ld4(dx0 + b + off[qq]);
            }
#define UNET_ROUTE(comp)                                                   \
    {                                                                      \
        float best = xv[0].comp;                                           \
        int arg = 0;                                                       \
        if (xv[1].comp > best) { best = xv[1].comp; arg = 1; }             \
        if (xv[2].comp > best) { best = xv[2].comp; arg = 2; }             \
        if (xv[3].comp > best) { best = xv[3].comp; arg = 3; }             \
        g[0].comp += arg == 0 ? acc.comp : 0.f;                            \
        g[1].comp += arg == 1 ? acc.comp : 0.f;                            \
        g[2].comp += arg == 2 ? acc.comp : 0.f;                            \
        g[3].comp += arg == 3 ? acc.comp : 0.f;                            \
    }
            UNET_ROUTE(x)
            UNET_ROUTE(y)
            UNET_ROUTE(z)
            UNET_ROUTE(w)
#undef UNET_ROUTE
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) st4(dx0 + b + off[qq], g[qq]);
            if constexpr (STATS) {
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) {
                    const float4 gm = make_float4(xv[qq].x > 0.f ? g[qq].x : 0.f, xv[qq].y > 0.f ? g[qq].y : 0.f,
                                                  xv[qq].z > 0.f ? g[qq].z : 0.f, xv[qq].w > 0.f ? g[qq].w : 0.f);
                    s1 = add4(s1, gm);
                    const float4 xh = make_float4((zr[qq].x - smu.x) * srs.x, (zr[qq].y - smu.y) * srs.y,
                                                  (zr[qq].z - smu.z) * srs.z, (zr[qq].w - smu.w) * srs.w);
                    s2 = fma4(gm, xh, s2);
                }
            }
        }
    }
    if constexpr (DWF) {  // the tile's [9][C] filter-gradient slab: the wave's columns by xor shuffles
        float4* R = T;    // (lanes l, l ^ QT, ...: one channel quad), then the four waves in order
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        __syncthreads();  // (every lane's window reads of T are done)
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            float4 s = fk[t];
#pragma unroll
            for (int o = QT; o < 64; o <<= 1) {
                s.x += __shfl_xor(s.x, o, 64);
                s.y += __shfl_xor(s.y, o, 64);
                s.z += __shfl_xor(s.z, o, 64);
                s.w += __shfl_xor(s.w, o, 64);
            }
            if (lane < QT) R[(wv * 9 + t) * QT + lane] = s;
        }
        __syncthreads();
        float* out = dwpart + (int64_t)tile * 9 * C;
        for (int e = threadIdx.x; e < 9 * QT; e += 256) {
            const int t = e / QT, qq = e - t * QT;
            const float4 s = add4(add4(R[t * QT + qq], R[(9 + t) * QT + qq]),
                                  add4(R[(18 + t) * QT + qq], R[(27 + t) * QT + qq]));
            st4(out + t * C + cbase + 4 * qq, s);
        }
    }
    if constexpr (STATS) {  // fixed-order reduction over the TW column lanes of each channel quad
        float* out = bnpart + (int64_t)tile * 2 * C;
        __syncthreads();
        T[threadIdx.x] = s1;
        __syncthreads();
        if (col == 0) {
            float4 t = T[q];
            for (int cl = 1; cl < G::TW; ++cl) t = add4(t, T[cl * QT + q]);
            st4(out + c, t);
        }
        __syncthreads();
        T[threadIdx.x] = s2;
        __syncthreads();
        if (col == 0) {
            float4 t = T[q];
            for (int cl = 1; cl < G::TW; ++cl) t = add4(t, T[cl * QT + q]);
            st4(out + C + c, t);
        }
    }
}

template <int MODE, bool DROP, int QT>
__global__ __launch_bounds__(256, 2) void dw_tile_bwd_filter(DView v, int N, int H, int W, int tiles_w, int tiles_h,
                                                          int ntiles, const float* __restrict__ dY,
                                                          float* __restrict__ part) {
    using G = Geom<QT>;
    __shared__ float4 T[G::NE];
    const int cbase = blockIdx.y * 4 * QT;
    const int C = v.C;
    const int q = threadIdx.x % QT, col = threadIdx.x / QT;
    const int c = cbase + 4 * q;
    float4 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f4(0.f);
    // XCD-contiguous assignment (as xcd_tile): XCD x walks tiles [x T/8, (x+1) T/8), its blocks
    // interleaved over that run, so neighbouring tiles' halos meet in one L2.  The block's slab and
    // the fixed-order slab sum stay as they were; only which tiles a slab sums changes
    const bool xo = (ntiles & 7) == 0 && (gridDim.x & 7) == 0;
    const int run = xo ? ntiles >> 3 : ntiles, base = xo ? (int)(blockIdx.x & 7) * run : 0;
    const int step = xo ? (int)(gridDim.x >> 3) : (int)gridDim.x;
    for (int i = xo ? (int)(blockIdx.x >> 3) : (int)blockIdx.x; i < run; i += step) {
        const int tile = base + i;
        int n, h0, w0;
        tile_coords(tile, tiles_w, tiles_h, G::TW, n, h0, w0);
        const int w = w0 + col;
        // the tile's 8 dy rows: issued with the halo loads (clamped addresses, masked on use)
        float4 gy[TH];
        const bool wok = w < W;
#pragma unroll
        for (int r = 0; r < TH; ++r) {
            const bool ok = wok && h0 + r < H;
            gy[r] = ld4(dY + (ok ? ((int64_t)(n * H + h0 + r) * W + w) * C + c : 0));
        }
        __syncthreads();  // previous tile's readers are done with T
        stage<MODE, DROP, QT>(T, v, n, h0, w0, H, W, cbase);
        __syncthreads();
        float4 a[3][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) a[i][j] = T[(i * G::HWp + col + j) * QT + q];
#pragma unroll
        for (int r = 0; r < TH; ++r) {
#pragma unroll
            for (int j = 0; j < 3; ++j) a[2][j] = T[((r + 2) * G::HWp + col + j) * QT + q];
            const float4 g = (wok && h0 + r < H) ? gy[r] : f4(0.f);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[i * 3 + j] = fma4(a[i][j], g, acc[i * 3 + j]);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                a[0][j] = a[1][j];
                a[1][j] = a[2][j];
            }
        }
    }
    // fixed-order reduction over the TW column lanes of each channel quad
    float* out = part + (int64_t)blockIdx.x * 9 * C;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        __syncthreads();
        T[threadIdx.x] = acc[t];
        __syncthreads();
        if (col == 0) {
            float4 s = T[q];
            for (int cl = 1; cl < G::TW; ++cl) s = add4(s, T[cl * QT + q]);
            st4(out + t * C + c, s);
        }
    }
}

int qt_for(int C) {
    if (C % 4) return 0;
    if (C % 64 == 0) return 16;  // (8 quads x 32 columns measured -0.6 % img/s, round 2)
    const int q = C / 4;
    return (q == 1 || q == 2 || q == 4 || q == 8) ? q : 0;
}

struct TilePlan {
    int qt, tw, tiles_w, tiles_h, chunks, ntiles, n;
};
TilePlan tile_plan(int N, int H, int W, int C) {
    TilePlan p;
    p.qt = qt_for(C);
    p.tw = p.qt ? 256 / p.qt : 1;
    p.tiles_w = (int)cdiv(W, p.tw);
    p.tiles_h = (int)cdiv(H, TH);
    p.chunks = p.qt ? C / (4 * p.qt) : 1;
    p.ntiles = N * p.tiles_w * p.tiles_h;
    p.n = N;
    return p;
}
int filter_blocks(const TilePlan& p) {
    // persistent blocks over all channel chunks: 1024 (~4 per CU), 512 at batch <= 8 (fewer slabs to
    // reduce; configs[4] batch 8 -0.8 %, configs[3] and batch 16 / 32 within the spread or slower with
    // 512, profiles/r5d_step_ab.txt d8_* / d16_* / dq_*)
    int target = lab_knob("UNET_DWF_BLOCKS", p.n <= lab_knob("UNET_DWF_SMALL_N", 8) ? 512 : 1024);
    if (target < 1) target = 1024;
    int g = (int)cdiv(target, p.chunks);
    if (g > p.ntiles) g = p.ntiles;
    if (g < 1) g = 1;
    return g;
}

#define UNET_TILE_DISPATCH_QT(KERNEL, MODE, DROP, GRID, ...)                       \
    switch (p.qt) {                                                                \
        case 16: KERNEL<MODE, DROP, 16><<<GRID, 256, tile_lds_pad, st>>>(__VA_ARGS__); break; \
        case 8: KERNEL<MODE, DROP, 8><<<GRID, 256, tile_lds_pad, st>>>(__VA_ARGS__); break;   \
        case 4: KERNEL<MODE, DROP, 4><<<GRID, 256, tile_lds_pad, st>>>(__VA_ARGS__); break;   \
        case 2: KERNEL<MODE, DROP, 2><<<GRID, 256, tile_lds_pad, st>>>(__VA_ARGS__); break;   \
        default: KERNEL<MODE, DROP, 1><<<GRID, 256, tile_lds_pad, st>>>(__VA_ARGS__); break;  \
    }
#define UNET_TILE_DISPATCH(KERNEL, GRID, ...)                                                       \
    switch (mode) {                                                                                 \
        case UNET_VIEW_PLAIN:                                                                       \
            if (drop) { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_PLAIN, true, GRID, __VA_ARGS__) }    \
            else { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_PLAIN, false, GRID, __VA_ARGS__) }        \
            break;                                                                                  \
        case UNET_VIEW_BNRELU:                                                                      \
            if (drop) { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_BNRELU, true, GRID, __VA_ARGS__) }   \
            else { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_BNRELU, false, GRID, __VA_ARGS__) }       \
            break;                                                                                  \
        case UNET_VIEW_POOL_BNRELU:                                                                 \
            if (drop) { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_POOL_BNRELU, true, GRID, __VA_ARGS__) } \
            else { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_POOL_BNRELU, false, GRID, __VA_ARGS__) }  \
            break;                                                                                  \
        default:                                                                                    \
            if (drop) { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_CONCAT, true, GRID, __VA_ARGS__) }   \
            else { UNET_TILE_DISPATCH_QT(KERNEL, UNET_VIEW_CONCAT, false, GRID, __VA_ARGS__) }       \
            break;                                                                                  \
    }

}  // namespace

bool dw_tiled_ok(int C) { return qt_for(C) != 0; }

int dw_tiled_fwd(const DView& v, int mode, bool drop, int N, int H, int W, const float* K, float* Y, hipStream_t st) {
    const unsigned tile_lds_pad = 0;
    TilePlan p = tile_plan(N, H, W, v.C);
    dim3 grid((unsigned)p.ntiles, (unsigned)p.chunks);
    UNET_TILE_DISPATCH(dw_tile_fwd, grid, v, N, H, W, p.tiles_w, p.tiles_h, K, Y)
    UNET_CHECK_LAUNCH("dwconv3x3_fwd(tiled)");
    return 0;
}

int dw_tiled_bwd_data(const DView& v, int mode, bool drop, int N, int H, int W, const float* K, const float* dY,
                      float* dx0, float* dx1, hipStream_t st) {
    const unsigned tile_lds_pad = 0;
    TilePlan p = tile_plan(N, H, W, v.C);
    dim3 grid((unsigned)p.ntiles, (unsigned)p.chunks);
    UNET_TILE_DISPATCH(dw_tile_bwd_data, grid, v, N, H, W, p.tiles_w, p.tiles_h, K, dY, dx0, dx1)
    UNET_CHECK_LAUNCH("dwconv3x3_bwd_data(tiled)");
    return 0;
}

int dw_tiled_bwd_data_bnstats(const DView& v, int mode, bool drop, int N, int H, int W, const float* K,
                              const float* dY, float* dx0, const float* mu, const float* rs, float* bnpart,
                              hipStream_t st, float* dwpart) {
    TilePlan p = tile_plan(N, H, W, v.C);
    dim3 grid((unsigned)p.ntiles, (unsigned)p.chunks);
    if (dwpart) {  // (BNRELU view, no dropout: checked by the caller)
#define UNET_DWF(Q)                                                                                         \
    dw_tile_bwd_data<UNET_VIEW_BNRELU, false, Q, true, true><<<grid, 256, 0, st>>>(v, N, H, W, p.tiles_w,   \
                                                                                    p.tiles_h, K, dY, dx0,   \
                                                                                    nullptr, mu, rs, bnpart, \
                                                                                    dwpart)
        switch (p.qt) {
            case 16: UNET_DWF(16); break;
            case 8: UNET_DWF(8); break;
            case 4: UNET_DWF(4); break;
            case 2: UNET_DWF(2); break;
            default: UNET_DWF(1); break;
        }
#undef UNET_DWF
        UNET_CHECK_LAUNCH("dwconv3x3_bwd_data_bnstats(tiled, filter gradient)");
        return 0;
    }
#define UNET_BNS(D, Q)                                                                                            \
    if (mode == UNET_VIEW_POOL_BNRELU)                                                                            \
        dw_tile_bwd_data<UNET_VIEW_POOL_BNRELU, D, Q, true><<<grid, 256, 0, st>>>(v, N, H, W, p.tiles_w, p.tiles_h, \
                                                                                  K, dY, dx0, nullptr, mu, rs, bnpart); \
    else                                                                                                          \
        dw_tile_bwd_data<UNET_VIEW_BNRELU, D, Q, true><<<grid, 256, 0, st>>>(v, N, H, W, p.tiles_w, p.tiles_h, K,   \
                                                                             dY, dx0, nullptr, mu, rs, bnpart)
#define UNET_BNS_QT(D)                      \
    switch (p.qt) {                          \
        case 16: UNET_BNS(D, 16); break;     \
        case 8: UNET_BNS(D, 8); break;       \
        case 4: UNET_BNS(D, 4); break;       \
        case 2: UNET_BNS(D, 2); break;       \
        default: UNET_BNS(D, 1); break;      \
    }
    if (drop) {
        UNET_BNS_QT(true)
    } else {
        UNET_BNS_QT(false)
    }
#undef UNET_BNS_QT
#undef UNET_BNS
    UNET_CHECK_LAUNCH("dwconv3x3_bwd_data_bnstats(tiled)");
    return 0;
}

size_t dw_tiled_ntiles(int N, int H, int W, int C) { return (size_t)tile_plan(N, H, W, C).ntiles; }

size_t dw_tiled_filter_partials(int N, int H, int W, int C) {
    TilePlan p = tile_plan(N, H, W, C);
    return (size_t)filter_blocks(p) * 9 * C;
}

int dw_tiled_bwd_filter(const DView& v, int mode, bool drop, int N, int H, int W, const float* dY, float* part,
                        int* S_out, hipStream_t st) {
    const unsigned tile_lds_pad = (unsigned)lab_knob("UNET_DWF_LDSPAD", 0);  // lab: dynamic LDS pad (fewer blocks per CU)
    TilePlan p = tile_plan(N, H, W, v.C);
    const int G = filter_blocks(p);
    dim3 grid((unsigned)G, (unsigned)p.chunks);
    UNET_TILE_DISPATCH(dw_tile_bwd_filter, grid, v, N, H, W, p.tiles_w, p.tiles_h, p.ntiles, dY, part)
    UNET_CHECK_LAUNCH("dwconv3x3_bwd_filter(tiled)");
    *S_out = G;
    return 0;
}

}  // namespace unet
