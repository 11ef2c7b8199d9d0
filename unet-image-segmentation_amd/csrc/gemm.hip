// FP32 MFMA GEMMs for the dense parts of the U-Net hot path (gfx950, v_mfma_f32_32x32x2_f32,
// exact f32: a k-ordered fmaf chain per output).
//
//   gemm_rows  : C[M, N] = A[M, K] . B[K, N]   rows = pixels (NHWC), B = a small weight matrix
//                  - pointwise half of SeparableConv2D fwd (model/u_net.py:14-20) with a
//                    BatchNorm-statistics epilogue (u_net.py:22-23),
//                  - its data gradient,
//                  - Conv2DTranspose(2, stride 2) fwd (u_net.py:88-94) as [M, Cin] x [Cin, 4 Cout]
//                    with a pixel-shuffle + bias epilogue (non-overlapping 2x2 taps),
//                  - Conv2DTranspose data gradient (pixel-unshuffle A operand).
//   gemm_wgrad : C[P, Q] = sum_m A[m, P] . B[m, Q]  (weight gradients, reduction over pixels),
//                split over m into slices; slices are summed in a fixed order (reduce_slabs),
//                so results are bitwise reproducible.
//
// Tiling (both kernels): 256 threads = 2x2 waves; each wave owns a (BM/2)x(BN/2) block of
// 32x32 MFMA tiles.  Operands are staged global -> registers -> LDS (k-major [BK][rows+4]
// images, so each MFMA operand fetch is one conflict-free ds_read_b32 per lane), double
// buffered: the next stage's global loads are in flight while the current stage's MFMAs run.
// The A operand passes through an activation view (BN+ReLU / dropout / unshuffle) on load.
#include <cstdlib>
#include "view.h"

namespace unet {

int colsum(const float* x, int64_t rows, int cols, float* out, void* ws, size_t ws_bytes, hipStream_t st);
size_t bn_partials_bytes(int64_t m, int c);
size_t colsum_workspace(int64_t rows, int cols);

namespace {

constexpr int BK = 16;

// A_BNBWD: A = dz of a BatchNorm + ReLU (+ dropout) output, formed on load from the incoming
// gradient da (a.src0) and the raw pre-BN z: g = da * drop * [z*sc+sh > 0],
// dz = sc * (g - p - (z - mu) * q) with per-channel (mu, p, q) = coef[0..3C) (see bn.hip).
enum { A_PLAIN = 0, A_BNRELU = 1, A_UNSHUFFLE = 2, A_BNBWD = 3 };
// E_BNPART: E_STORE, and the stored C is the complete da of a BatchNorm + ReLU block whose raw
// z is g.z (same [M][N] layout): the tile also emits that block's BN-backward partial sums
// bnpart[tile][0][n] = sum g, bnpart[tile][1][n] = sum g * xhat, g = da * [z*sc+sh > 0],
// xhat = (z - mu) * rs (the dwtile.hip STATS format, finished by unet_bn_relu_bwd_stats_finish).
enum { E_STORE = 0, E_STATS = 1, E_SHUFFLE = 2, E_BNPART = 3 };

struct RowsArgs {
    DView a;  // A operand: PLAIN/BNRELU -> a.src0[m * a.c0 + k]; UNSHUFFLE -> a.src0 = dU
    int64_t M;
    int K;
    int uH, uW, uf;  // UNSHUFFLE: m = (n, i, j) over uH x uW, dU is (n, 2uH, 2uW, uf)
    const float* B;
    int64_t sbk, sbn;
    int N;
    float* C;
    int64_t ldc;
    const float* bias;
    float2* stats;
    int sH, sW, sf;  // SHUFFLE epilogue: m = (n, i, j) over sH x sW, out (n, 2sH, 2sW, sf)
    const float* z;     // A_BNBWD: pre-BN z (same layout as a.src0)
    const float* coef;  // A_BNBWD: (mu, p, q) x C
    float* side;        // A_BNBWD: optional copy of the formed A (= dz), written by N-tile 0
    const float *bsc, *bsh, *bmu, *brs;  // E_BNPART: per-column BN scale/shift, mean/rstd (NULL: no xhat)
    float* bnpart;                       // E_BNPART: [cdiv(M, BM)][2][N] partial sums, one slab per row tile
                                         //   (BM = 64 or 128, convt_bnpart_bm; sized by the _slabs query)
    float ep_rate, ep_inv_keep;          // E_BNPART: dropout between the block and C's consumer (rate 0: none);
    uint64_t ep_seed;                    //   g also carries the mask of element (m, n) (common.h drop_mult)
    int ko;  // lab build only (UNET_ROWS_KO): knock-out bits for timing decompositions, else 0
    const unsigned short* Bx;  // split-precision route: B as three bf16 planes [3][N][K] (k contiguous), or NULL
};
#ifdef UNET_LAB_BUILD
#define ROWS_KO(g, bit) (((g).ko & (bit)) != 0)
#else
#define ROWS_KO(g, bit) false
#endif

__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

// XCD-aware placement: workgroups go to the 8 XCDs round-robin by linear id (x fastest), and each
// XCD has its own L2.  For a (groups x sibs) grid whose sibling blocks read the same operand rows
// (the N-tiles of one row tile, the (p, q) tiles of one m-slice), renumber the linear id so that
// all siblings of a group run on one XCD and share those rows through its L2 instead of each
// fetching them from HBM.  Needs groups % 8 == 0 (else the grid order is kept); same tiles, same
// arithmetic -- only where each tile runs changes.  grid x = groups, y = sibs.
__device__ __forceinline__ void xcd_group_order(int groups, int sibs, int& grp, int& sib) {
    grp = blockIdx.x;
    sib = blockIdx.y;
    if (sibs > 1 && (groups & 7) == 0) {
        const int L = blockIdx.x + blockIdx.y * groups, u = L >> 3;
        grp = (u / sibs) * 8 + (L & 7);
        sib = u % sibs;
    }
}
// the same with the siblings along grid x (the weight-gradient GEMMs: x = (p, q) tile, y = m-slice)
__device__ __forceinline__ void xcd_group_order_sx(int sibs, int groups, int& sib, int& grp) {
    sib = blockIdx.x;
    grp = blockIdx.y;
    if (sibs > 1 && (groups & 7) == 0) {
        const int L = blockIdx.x + blockIdx.y * sibs, u = L >> 3;
        grp = (u / sibs) * 8 + (L & 7);
        sib = u % sibs;
    }
}

template <int BM, int BN, int AMODE, bool DROP, int EPI>
__global__ __launch_bounds__(256) void gemm_rows_kernel(RowsArgs g) {
    constexpr int LDA = BM + 4, LDB = BN + 4;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int AR = BM / 16;  // A elements per thread per stage
    constexpr int BR = BN / 16;  // B elements per thread per stage
    __shared__ float As[2][BK][LDA];
    __shared__ float Bs[2][BK][LDB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lo = lane & 31, hi = lane >> 5;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int M_rem = (int)((g.M - m0) < BM ? (g.M - m0) : BM);

    // ---- A staging geometry: k-lane ak, rows arow0 + 16 r
    const int ak = tid & 15;
    const int arow0 = tid >> 4;
    int aoff[AR];
#pragma unroll
    for (int r = 0; r < AR; ++r) {
        const int rr = arow0 + 16 * r;
        if (rr < M_rem) {
            const int64_t m = m0 + rr;
            if constexpr (AMODE == A_UNSHUFFLE) {
                const int64_t hw = (int64_t)g.uH * g.uW;
                const int n = (int)(m / hw);
                const int rem = (int)(m - (int64_t)n * hw);
                const int i = rem / g.uW, j = rem - (rem / g.uW) * g.uW;
                aoff[r] = ((n * 2 * g.uH + 2 * i) * 2 * g.uW + 2 * j) * g.uf;
            } else {
                aoff[r] = (int)(m * g.a.c0);
            }
        } else {
            aoff[r] = -1;
        }
    }
    // ---- B staging geometry
    const bool bkc = g.sbk == 1;
    int bk_[BR], bn_[BR];
#pragma unroll
    for (int r = 0; r < BR; ++r) {
        if (bkc) {
            bk_[r] = tid & 15;
            bn_[r] = (tid >> 4) + 16 * r;
        } else {
            bn_[r] = tid % BN;
            bk_[r] = tid / BN + (256 / BN) * r;
        }
    }

    float ra[AR], rb[BR];
    auto load_stage = [&](int k0) {
        const int k = k0 + ak;
        const bool kv = k < g.K;
        int koff = k;
        float sc = 1.f, sh = 0.f;
        if constexpr (AMODE == A_UNSHUFFLE) {
            const int ab = k / g.uf;
            const int co = k - ab * g.uf;
            koff = (ab >> 1) * (2 * g.uW * g.uf) + (ab & 1) * g.uf + co;
        }
        if constexpr (AMODE == A_BNRELU) {
            if (kv) {
                sc = g.a.sc0[k];
                sh = g.a.sh0[k];
            }
        }
#pragma unroll
        for (int r = 0; r < AR; ++r) {
            float v = 0.f;
            if (kv && aoff[r] >= 0) {
                v = g.a.src0[aoff[r] + koff];
                if constexpr (AMODE == A_BNRELU) v = bnrelu(v, sc, sh);
                if constexpr (DROP)
                    v *= drop_mult(g.a.seed, (uint64_t)(m0 + arow0 + 16 * r) * g.a.C + k, g.a.rate, g.a.inv_keep);
            }
            ra[r] = v;
        }
#pragma unroll
        for (int r = 0; r < BR; ++r) {
            const int kk = k0 + bk_[r], nn = n0 + bn_[r];
            rb[r] = (kk < g.K && nn < g.N) ? g.B[kk * g.sbk + nn * g.sbn] : 0.f;
        }
    };
    auto store_stage = [&](int buf) {
#pragma unroll
        for (int r = 0; r < AR; ++r) As[buf][ak][arow0 + 16 * r] = ra[r];
#pragma unroll
        for (int r = 0; r < BR; ++r) Bs[buf][bk_[r]][bn_[r]] = rb[r];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

    const int nk = (g.K + BK - 1) / BK;
    load_stage(0);
    store_stage(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_stage((kt + 1) * BK);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            float av[TM], bv[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) av[tm] = As[buf][2 * kk + hi][wm * (BM / 2) + tm * 32 + lo];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) bv[tn] = Bs[buf][2 * kk + hi][wn * (BN / 2) + tn * 32 + lo];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[tm], bv[tn], acc[tm][tn], 0, 0, 0);
        }
        if (kt + 1 < nk) store_stage(buf ^ 1);
        __syncthreads();
    }

    // ---------------------------------------------------------------- epilogue
    if constexpr (EPI == E_STORE || EPI == E_STATS) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * (BN / 2) + tn * 32 + lo;
                if (n >= g.N) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = wm * (BM / 2) + tm * 32 + acc_row(r, hi);
                    if (rr < M_rem) g.C[(m0 + rr) * g.ldc + n] = acc[tm][tn][r];
                }
            }
    }
    if constexpr (EPI == E_STATS) {
        // per-column (count, mean, M2) over this block's valid rows: two passes in registers
        float* red = &As[0][0][0];
        float mean[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * (BN / 2) + tn * 32 + lo;
            float s = 0.f;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (wm * (BM / 2) + tm * 32 + acc_row(r, hi) < M_rem) s += acc[tm][tn][r];
            s += __shfl_xor(s, 32, 64);
            if (hi == 0) red[wm * BN + col] = s;
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * (BN / 2) + tn * 32 + lo;
            mean[tn] = (red[col] + red[BN + col]) / (float)M_rem;
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * (BN / 2) + tn * 32 + lo;
            float q = 0.f;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (wm * (BM / 2) + tm * 32 + acc_row(r, hi) < M_rem) {
                        const float d = acc[tm][tn][r] - mean[tn];
                        q = fmaf(d, d, q);
                    }
            q += __shfl_xor(q, 32, 64);
            if (hi == 0) red[wm * BN + col] = q;
        }
        __syncthreads();
        if (wm == 0 && hi == 0) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = wn * (BN / 2) + tn * 32 + lo;
                const int n = n0 + col;
                if (n < g.N) g.stats[(int64_t)blockIdx.x * g.N + n] = make_float2(mean[tn], red[col] + red[BN + col]);
            }
        }
    }
    if constexpr (EPI == E_SHUFFLE) {
        const int64_t hw = (int64_t)g.sH * g.sW;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * (BN / 2) + tn * 32 + lo;
            if (n >= g.N) continue;
            const int ab = n / g.sf;
            const int co = n - ab * g.sf;
            const int a = ab >> 1, b = ab & 1;
            const float bias = g.bias ? g.bias[co] : 0.f;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = wm * (BM / 2) + tm * 32 + acc_row(r, hi);
                    if (rr >= M_rem) continue;
                    const int64_t m = m0 + rr;
                    const int img = (int)(m / hw);
                    const int rem = (int)(m - img * hw);
                    const int i = rem / g.sW, j = rem - (rem / g.sW) * g.sW;
                    const int64_t o = ((int64_t)(img * 2 * g.sH + 2 * i + a) * (2 * g.sW) + 2 * j + b) * g.sf + co;
                    g.C[o] = acc[tm][tn][r] + bias;
                }
        }
    }
}

// --------------------------------------------------------------------------------- wgrad ----
// W_BNBWD (B operand, vectorised kernel only): B = dz of a BatchNorm + ReLU output formed on load
// from da (b.src0) and the raw z exactly as A_BNBWD does (coef = (mu, p, q)), so the data-gradient
// GEMM need not store dz for this kernel.
enum { W_PLAIN = 0, W_BNRELU = 1, W_UNSHUFFLE = 2, W_BNBWD = 3 };

struct WgradArgs {
    DView a;
    int P;
    int uH, uW, uf;  // A UNSHUFFLE geometry (m over uH x uW, dU (n, 2uH, 2uW, uf))
    DView b;
    int Q;
    int64_t M, mslice;
    float* slab;  // [S][P][Q]
    const float* bz;     // W_BNBWD: raw z (same layout as b.src0)
    const float* bcoef;  // W_BNBWD: (mu, p, q) x Q
    float* colpart;      // optional [S][P]: column sums of A over the block's m slice (vectorised kernel, q-tile 0)
    bool x6;             // 128 x 128 tiles take the split-precision (bf16x6) kernel
};

template <int BP, int BQ, int AMODE, bool ADROP, int BMODE, bool BDROP>
__global__ __launch_bounds__(256) void gemm_wgrad_kernel(WgradArgs g) {
    constexpr int LDA = BP + 4, LDB = BQ + 4;
    constexpr int TM = BP / 64, TN = BQ / 64;
    constexpr int AR = BP / 16, BR = BQ / 16;
    constexpr int AS = 256 / BP, BS = 256 / BQ;  // row steps between a thread's staged elements
    __shared__ float As[2][BK][LDA];
    __shared__ float Bs[2][BK][LDB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wp = wave >> 1, wq = wave & 1;
    const int lo = lane & 31, hi = lane >> 5;
    const int ntp = (g.P + BP - 1) / BP;
    const int p0 = (blockIdx.x % ntp) * BP;
    const int q0 = (blockIdx.x / ntp) * BQ;
    const int64_t mb = (int64_t)blockIdx.y * g.mslice;
    const int64_t me = mb + g.mslice < g.M ? mb + g.mslice : g.M;

    // A: this thread stages column p = p0 + ap, rows amm + AS*r of each stage
    const int ap = tid % BP, amm = tid / BP;
    const int p = p0 + ap;
    const bool pv = p < g.P;
    float asc = 1.f, ash = 0.f;
    int poff = p;
    if constexpr (AMODE == W_BNRELU) {
        if (pv) {
            asc = g.a.sc0[p];
            ash = g.a.sh0[p];
        }
    }
    if constexpr (AMODE == W_UNSHUFFLE) {
        const int ab = p / g.uf;
        const int co = p - ab * g.uf;
        poff = (ab >> 1) * (2 * g.uW * g.uf) + (ab & 1) * g.uf + co;
    }
    const int bq = tid % BQ, bmm = tid / BQ;
    const int q = q0 + bq;
    const bool qv = q < g.Q;
    float bsc = 1.f, bsh = 0.f;
    if constexpr (BMODE == W_BNRELU) {
        if (qv) {
            bsc = g.b.sc0[q];
            bsh = g.b.sh0[q];
        }
    }

    float ra[AR], rb[BR];
    auto load_stage = [&](int64_t k0) {
#pragma unroll
        for (int r = 0; r < AR; ++r) {
            const int64_t m = k0 + amm + AS * r;
            float v = 0.f;
            if (pv && m < me) {
                if constexpr (AMODE == W_UNSHUFFLE) {
                    const int64_t hw = (int64_t)g.uH * g.uW;
                    const int n = (int)(m / hw);
                    const int rem = (int)(m - n * hw);
                    const int i = rem / g.uW, j = rem - (rem / g.uW) * g.uW;
                    v = g.a.src0[(int64_t)((n * 2 * g.uH + 2 * i) * 2 * g.uW + 2 * j) * g.uf + poff];
                } else {
                    v = g.a.src0[m * g.a.c0 + p];
                    if constexpr (AMODE == W_BNRELU) v = bnrelu(v, asc, ash);
                    if constexpr (ADROP) v *= drop_mult(g.a.seed, (uint64_t)m * g.a.C + p, g.a.rate, g.a.inv_keep);
                }
            }
            ra[r] = v;
        }
#pragma unroll
        for (int r = 0; r < BR; ++r) {
            const int64_t m = k0 + bmm + BS * r;
            float v = 0.f;
            if (qv && m < me) {
                v = g.b.src0[m * g.b.c0 + q];
                if constexpr (BMODE == W_BNRELU) v = bnrelu(v, bsc, bsh);
                if constexpr (BDROP) v *= drop_mult(g.b.seed, (uint64_t)m * g.b.C + q, g.b.rate, g.b.inv_keep);
            }
            rb[r] = v;
        }
    };
    auto store_stage = [&](int buf) {
#pragma unroll
        for (int r = 0; r < AR; ++r) As[buf][amm + AS * r][ap] = ra[r];
#pragma unroll
        for (int r = 0; r < BR; ++r) Bs[buf][bmm + BS * r][bq] = rb[r];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

    const int nk = (int)((me - mb + BK - 1) / BK);
    if (nk > 0) {
        load_stage(mb);
        store_stage(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_stage(mb + (int64_t)(kt + 1) * BK);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            float av[TM], bv[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) av[tm] = As[buf][2 * kk + hi][wp * (BP / 2) + tm * 32 + lo];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) bv[tn] = Bs[buf][2 * kk + hi][wq * (BQ / 2) + tn * 32 + lo];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[tm], bv[tn], acc[tm][tn], 0, 0, 0);
        }
        if (kt + 1 < nk) store_stage(buf ^ 1);
        __syncthreads();
    }
    float* slab = g.slab + (int64_t)blockIdx.y * g.P * g.Q;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int qq = q0 + wq * (BQ / 2) + tn * 32 + lo;
            if (qq >= g.Q) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int pp = p0 + wp * (BP / 2) + tm * 32 + acc_row(r, hi);
                if (pp < g.P) slab[(int64_t)pp * g.Q + qq] = acc[tm][tn][r];
            }
        }
}

// ---------------------------------------------------------------- vectorised rows GEMM ----
// As[m][BK+4], Bs[n][BK+4] (k contiguous).  In a group of 8 k, MFMA step s takes k-slot 0 =
// k0+s and k-slot 1 = k0+4+s, so lane (row, half) feeds 4 consecutive MFMAs from ONE
// ds_read_b128 of its row.  Row stride BK+4 floats makes those reads conflict-free.
//
// X6 (split precision, see common.h split4 / mfma_x6): the staged A values are split into three
// bf16 planes as they are written to LDS ([row][k] images, k contiguous, row stride BK + 8 bf16 =
// conflict-free ds_read_b128); B arrives pre-split (g.Bx, [3][N][K] planes written once per weight
// update by unet_split_x3_ex) and is copied 16 bytes at a time.  Every 16-deep k step runs the six
// v_mfma_f32_32x32x16_bf16 of mfma_x6 per 32x32 tile: 6 x 32 cycles instead of the 8 x 64 of
// v_mfma_f32_32x32x2_f32, at fp32 accuracy.  The bf16 MFMA leaves 24 of its 32 issue cycles to
// VALU (the f32 MFMA shares the FP32 vector datapath), so the BN-backward operand transform and
// the split hide under the matrix work.  With 2.7x fewer matrix cycles per stage the load latency
// is what a stage must cover: X6 stages BK = 32 in ONE LDS buffer (61 KB at 128 x 128: two blocks
// per CU), loads of stage k+1 in registers while stage k computes, two barriers per stage (the
// co-resident block's MFMAs fill the store phase).  Loads, operand views and epilogues are shared.
#ifdef UNET_LAB_BUILD
// lab: ko bits 8-15 = stagger (that many s_sleep 32, ~2048 cycles each) for the second half of the
// grid's blocks (bit 16: the odd blocks instead), so the two blocks sharing a CU do not run in lockstep
__device__ __forceinline__ void lab_stagger(int ko) {
    const int n = (ko >> 8) & 255;
    if (n == 0) return;
    const unsigned lin = blockIdx.x + blockIdx.y * gridDim.x, tot = gridDim.x * gridDim.y;
    const bool late = (ko & 0x10000) ? (lin & 1) : (lin >= tot / 2);
    if (late)
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(32);
}
#define ROWS_STAGGER(g) lab_stagger((g).ko)
// lab: ko bit 17 = per-block stamps into lab_rows_stamps[block][4] (thread 0 only): s_memrealtime
// (100 MHz, device-wide) at start and end, s_memtime (shader cycles, per XCD) after the prologue
// stage and after the k-loop
__device__ unsigned long long lab_rows_stamps[65536 * 4];
#define ROWS_STAMP(g, i)                                                                       \
    do {                                                                                       \
        if (((g).ko & 0x20000) && threadIdx.x == 0) {                                          \
            const unsigned lin_ = blockIdx.x + blockIdx.y * gridDim.x;                         \
            if (lin_ < 65536) lab_rows_stamps[4 * lin_ + (i)] =                               \
                ((i) == 0 || (i) == 3) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime(); \
        }                                                                                      \
    } while (0)
#else
#define ROWS_STAGGER(g) ((void)0)
#define ROWS_STAMP(g, i) ((void)0)
#endif

template <int BM, int BN, int BK, int AMODE, bool DROP, int EPI, bool BKC, bool X6 = false>
__global__ __launch_bounds__(256, X6 ? 2 : 1) void gemm_rows_vec(RowsArgs g) {
    main_stream_prio();
    ROWS_STAGGER(g);
    ROWS_STAMP(g, 0);
    constexpr int LR = BK + 4;     // A (and k-contiguous B) LDS row stride, floats
    constexpr int LB = BN + 4;     // k-major B LDS row stride (n-contiguous weights)
    constexpr int XR = BK + 8;     // X6: bf16 row stride of the split planes
    constexpr int KQ = BK / 4;
    constexpr int NQ = BN / 4;
    constexpr int AQ = BM * KQ / 256;
    constexpr int BQ = BN * KQ / 256;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int BSZ = BKC ? BN * LR : BK * LB;
    constexpr int F32_BYTES = 4 * 2 * (BM * LR + BSZ);
    // X6 + BatchNorm backward: the five per-channel operand vectors (scale, shift, mu, p, q) of all
    // K <= X6_KMAX channels sit in LDS (read per stage), not in 20 live registers across the k-loop
    constexpr int X6_KMAX = 512;
    constexpr bool XCOEF = X6 && AMODE == A_BNBWD;
    constexpr int X6_BYTES = 2 * 3 * (BM + BN) * XR + (XCOEF ? 4 * 5 * X6_KMAX : 0);  // one buffer
    static_assert(!X6 || BK == 32, "X6 rows GEMM: 32-deep stages");
    __shared__ __attribute__((aligned(16))) char smem[X6 ? X6_BYTES : F32_BYTES];
    float* xcoef = reinterpret_cast<float*>(smem + 2 * 3 * (BM + BN) * XR);  // XCOEF: [5][X6_KMAX]
    // fp32 images (the X6 path uses the first bytes of As as epilogue scratch only)
    float (*As)[BM * LR] = reinterpret_cast<float (*)[BM * LR]>(smem);
    float (*Bs)[BSZ] = reinterpret_cast<float (*)[BSZ]>(smem + 4 * 2 * BM * LR);
    // X6 planes: Ax[plane * BM + row][k], Bx[plane * BN + col][k]
    unsigned short* Ax = reinterpret_cast<unsigned short*>(smem);
    unsigned short* Bx = Ax + 3 * BM * XR;
    // X6: B chunks (8 bf16 of one plane row) per thread and stage
    constexpr int XCH = BK / 8, XQ = 3 * BN * XCH / 256;
    static_assert(!X6 || (3 * BN * XCH) % 256 == 0, "X6: whole B chunks per thread");

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lo = lane & 31, hi = lane >> 5;
    int mt, nt;  // row tile, column tile (the N-tiles of a row tile share its A rows through one L2)
    xcd_group_order(gridDim.x, gridDim.y, mt, nt);
    const int m0 = mt * BM;
    const int n0 = nt * BN;
    const int M_rem = (g.M - m0) < BM ? (int)(g.M - m0) : BM;
    const int K = g.K;

    // A: this thread stages k-quad kq of rows arow + (256/KQ) r
    const int kq = tid % KQ;
    const int arow = tid / KQ;
    int aoff[AQ];
#pragma unroll
    for (int r = 0; r < AQ; ++r) {
        const int rr = arow + (256 / KQ) * r;
        if (rr < M_rem) {
            const int m = m0 + rr;
            if constexpr (AMODE == A_UNSHUFFLE) {  // (0, 0) tap of pixel m: dU row 2 (m / uW), column 2 (m % uW)
                const int ur = m / g.uW;
                aoff[r] = (4 * ur * g.uW + 2 * (m - ur * g.uW)) * g.uf;
            } else {
                aoff[r] = m * g.a.c0;
            }
        } else {
            aoff[r] = -1;
        }
    }
    // B: per-thread element offsets at k0 = 0 (-1: column out of range); k advances by sbk
    const int sbk = (int)g.sbk, sbn = (int)g.sbn;
    const int bq_k = BKC ? tid % KQ : tid / NQ;      // k-quad (BKC) or k-row (n-contiguous)
    const int bq_n = BKC ? tid / KQ : tid % NQ;      // column (BKC) or n-quad
    int boff[BQ];
#pragma unroll
    for (int r = 0; r < BQ; ++r) {
        if constexpr (BKC) {
            const int n = n0 + bq_n + (256 / KQ) * r;
            boff[r] = n < g.N ? n * sbn + 4 * bq_k : -1;
        } else {
            const int n = n0 + 4 * bq_n;
            boff[r] = n < g.N ? (bq_k + (256 / NQ) * r) * sbk + n : -1;
        }
    }

    // Loads are issued unconditionally from clamped addresses; validity masks, the view
    // transform and dropout are applied when the registers are written to LDS, so no load is
    // waited for before the stage's MFMAs.
    float4 ra[AQ], rb[BQ];
    float4 rz[AMODE == A_BNBWD ? AQ : 1];
    float4 csc, csh, cmu, cp, cq;  // per-stage channel constants of this thread's k-quad
    int ak = 0;                    // k of this thread's A quad in the staged k-stage
    bool bok[BQ];
    uint4 rx[X6 ? XQ : 1];        // X6: staged B plane chunks
    bool xok[X6 ? XQ : 1];
    int xoff[X6 ? XQ : 1], xlds[X6 ? XQ : 1];  // chunk's plane-row element offset at k0 = 0 (-1: out of range) / LDS slot
    if constexpr (X6) {
        const int64_t plane = (int64_t)g.N * K;
#pragma unroll
        for (int j = 0; j < XQ; ++j) {
            const int c = tid + 256 * j;
            const int p = c / (BN * XCH), rem = c - p * (BN * XCH);
            const int row = rem / XCH, kc = rem - row * XCH;
            const int n = n0 + row;
            xoff[j] = n < g.N ? (int)(p * plane + (int64_t)n * K) + 8 * kc : -1;
            xlds[j] = (p * BN + row) * XR + 8 * kc;
        }
    }
    auto load_stage = [&](int k0) {
        const int k = k0 + 4 * kq;
        ak = k;
        if (k0 > 0 && ROWS_KO(g, 4)) return;  // lab: no k-loop operand loads
        const int kc = k < K ? k : 0;
        int koff = kc;
        if constexpr (AMODE == A_UNSHUFFLE) {
            const int ab = kc / g.uf;
            const int co = kc - ab * g.uf;
            koff = (ab >> 1) * (2 * g.uW * g.uf) + (ab & 1) * g.uf + co;
        }
        if constexpr ((AMODE == A_BNRELU || AMODE == A_BNBWD) && !XCOEF) {
            csc = ld4(g.a.sc0 + kc);
            csh = ld4(g.a.sh0 + kc);
        }
        if constexpr (AMODE == A_BNBWD && !XCOEF) {
            cmu = ld4(g.coef + kc);
            cp = ld4(g.coef + K + kc);
            cq = ld4(g.coef + 2 * K + kc);
        }
#pragma unroll
        for (int r = 0; r < AQ; ++r) {
            const int o = (aoff[r] < 0 ? 0 : aoff[r]) + koff;
            ra[r] = ld4(g.a.src0 + o);
            if constexpr (AMODE == A_BNBWD) rz[r] = ld4(g.z + o);
        }
        if constexpr (X6) {
#pragma unroll
            for (int j = 0; j < XQ; ++j) {  // (K % BK == 0 on this route: every chunk's k exists)
                xok[j] = xoff[j] >= 0;
                rx[j] = *reinterpret_cast<const uint4*>(g.Bx + (xok[j] ? xoff[j] + k0 : 0));
            }
        } else {
#pragma unroll
        for (int r = 0; r < BQ; ++r) {
            const int kk = BKC ? k0 + 4 * bq_k : k0 + bq_k + (256 / NQ) * r;
            bok[r] = boff[r] >= 0 && kk < K;
            rb[r] = ld4(g.B + (bok[r] ? boff[r] + (BKC ? k0 : k0 * sbk) : 0));
        }
        }
    };
    auto store_stage = [&](int buf) {
        const bool kv = ak < K;
        if constexpr (XCOEF) {  // (ak < K on this route: K % 32 == 0)
            csc = *reinterpret_cast<const float4*>(xcoef + ak);
            csh = *reinterpret_cast<const float4*>(xcoef + X6_KMAX + ak);
            cmu = *reinterpret_cast<const float4*>(xcoef + 2 * X6_KMAX + ak);
            cp = *reinterpret_cast<const float4*>(xcoef + 3 * X6_KMAX + ak);
            cq = *reinterpret_cast<const float4*>(xcoef + 4 * X6_KMAX + ak);
        }
#pragma unroll
        for (int r = 0; r < AQ; ++r) {
            float4 v = ra[r];
            if constexpr (AMODE == A_BNRELU) v = bnrelu4(v, csc, csh);
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)(m0 + arow + (256 / KQ) * r) * g.a.C + (kv ? ak : 0);
                v = mul4(v, drop_mult4(g.a.seed, i, g.a.rate, g.a.inv_keep));
            }
            if constexpr (AMODE == A_BNBWD) {
                const float4 zz = rz[r];
                v.x = fmaf(zz.x, csc.x, csh.x) > 0.f ? v.x : 0.f;
                v.y = fmaf(zz.y, csc.y, csh.y) > 0.f ? v.y : 0.f;
                v.z = fmaf(zz.z, csc.z, csh.z) > 0.f ? v.z : 0.f;
                v.w = fmaf(zz.w, csc.w, csh.w) > 0.f ? v.w : 0.f;
                v.x = csc.x * (v.x - cp.x - (zz.x - cmu.x) * cq.x);
                v.y = csc.y * (v.y - cp.y - (zz.y - cmu.y) * cq.y);
                v.z = csc.z * (v.z - cp.z - (zz.z - cmu.z) * cq.z);
                v.w = csc.w * (v.w - cp.w - (zz.w - cmu.w) * cq.w);
            }
            if (!kv || aoff[r] < 0) v = f4(0.f);
            if constexpr (AMODE == A_BNBWD) {
                if (g.side && nt == 0 && kv && aoff[r] >= 0 && !ROWS_KO(g, 2)) st4(g.side + aoff[r] + ak, v);
            }
            const int row = arow + (256 / KQ) * r;
            if constexpr (X6) {
                const Split4 sp = split4(v);
                unsigned short* d = Ax + row * XR + 4 * kq;
                *reinterpret_cast<uint2*>(d) = sp.h;
                *reinterpret_cast<uint2*>(d + BM * XR) = sp.m;
                *reinterpret_cast<uint2*>(d + 2 * BM * XR) = sp.l;
            } else {
                *reinterpret_cast<float4*>(&As[buf][row * LR + 4 * kq]) = v;
            }
        }
        if constexpr (X6) {
#pragma unroll
            for (int j = 0; j < XQ; ++j)
                *reinterpret_cast<uint4*>(Bx + xlds[j]) = xok[j] ? rx[j] : make_uint4(0u, 0u, 0u, 0u);
            return;
        }
#pragma unroll
        for (int r = 0; r < BQ; ++r) {
            const float4 v = bok[r] ? rb[r] : f4(0.f);
            if constexpr (BKC) {
                *reinterpret_cast<float4*>(&Bs[buf][(bq_n + (256 / KQ) * r) * LR + 4 * bq_k]) = v;
            } else {
                *reinterpret_cast<float4*>(&Bs[buf][(bq_k + (256 / NQ) * r) * LB + 4 * bq_n]) = v;
            }
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

    const int nk = (K + BK - 1) / BK;
    if constexpr (XCOEF) {
        for (int i = tid; i < K; i += 256) {
            xcoef[i] = g.a.sc0[i];
            xcoef[X6_KMAX + i] = g.a.sh0[i];
            xcoef[2 * X6_KMAX + i] = g.coef[i];
            xcoef[3 * X6_KMAX + i] = g.coef[K + i];
            xcoef[4 * X6_KMAX + i] = g.coef[2 * K + i];
        }
    }
    load_stage(0);
    if constexpr (XCOEF) __syncthreads();
    store_stage(0);
    __syncthreads();
    ROWS_STAMP(g, 1);
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_stage((kt + 1) * BK);
        if constexpr (X6) {
#pragma unroll
            for (int ks = 0; ks < BK / 16; ++ks) {
                // the wave's B fragments for this 16-deep step, then one row tile's A fragments at a
                // time (36 operand registers instead of 48)
                bf16x8 bfr[TN][3];
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        bfr[tn][p] = *reinterpret_cast<const bf16x8*>(
                            Bx + (p * BN + wn * (BN / 2) + tn * 32 + lo) * XR + ks * 16 + 8 * hi);
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    bf16x8 af[3];
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        af[p] = *reinterpret_cast<const bf16x8*>(
                            Ax + (p * BM + wm * (BM / 2) + tm * 32 + lo) * XR + ks * 16 + 8 * hi);
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_x6(af, bfr[tn], acc[tm][tn]);
                }
            }
            // one buffer: every wave's fragment reads are done before the next stage overwrites it
            __syncthreads();
            if (kt + 1 < nk) {
                store_stage(0);
                __syncthreads();
            }
            continue;
        } else {
#pragma unroll
        for (int kg = 0; kg < BK / 8; ++kg) {
            float4 af[TM], bf[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
                af[tm] = *reinterpret_cast<const float4*>(&As[buf][(wm * (BM / 2) + tm * 32 + lo) * LR + kg * 8 + 4 * hi]);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = wn * (BN / 2) + tn * 32 + lo;
                if constexpr (BKC) {
                    bf[tn] = *reinterpret_cast<const float4*>(&Bs[buf][col * LR + kg * 8 + 4 * hi]);
                } else {
                    const float* bp = &Bs[buf][(kg * 8 + 4 * hi) * LB + col];
                    bf[tn] = make_float4(bp[0], bp[LB], bp[2 * LB], bp[3 * LB]);
                }
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].x, bf[tn].x, acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].y, bf[tn].y, acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].z, bf[tn].z, acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm].w, bf[tn].w, acc[tm][tn], 0, 0, 0);
                }
        }
        }
        if (kt + 1 < nk) store_stage(buf ^ 1);
        __syncthreads();
    }

    ROWS_STAMP(g, 2);
    const bool full = M_rem == BM;  // every row of the tile exists: no per-row checks
    if constexpr (EPI == E_STORE || EPI == E_STATS || EPI == E_BNPART) {
        const int ldc = (int)g.ldc;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * (BN / 2) + tn * 32 + lo;
                if (n >= g.N) continue;
                const int rb0 = wm * (BM / 2) + tm * 32 + 4 * hi;  // acc_row(r, hi) = rb0 + acc_row(r, 0)
                float* cp = g.C + (int64_t)(m0 + rb0) * g.ldc + n;
                if (ROWS_KO(g, 1)) continue;  // lab: no C stores
                if (full) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) cp[acc_row(r, 0) * ldc] = acc[tm][tn][r];
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (rb0 + acc_row(r, 0) < M_rem) cp[acc_row(r, 0) * ldc] = acc[tm][tn][r];
                }
            }
    }
    if constexpr (EPI == E_STATS) {
        // Per-wave (mean, M2) over its BM/2 rows, then one Chan combine of the two row-halves
        // (one barrier); the partial is the (mean, M2) of the tile's M_rem rows.
        float2* red = reinterpret_cast<float2*>(&As[0][0]);
        const int wr0 = wm * (BM / 2);
        const int cnt = M_rem - wr0 < 0 ? 0 : (M_rem - wr0 < BM / 2 ? M_rem - wr0 : BM / 2);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * (BN / 2) + tn * 32 + lo;
            float s = 0.f;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (full || wr0 + tm * 32 + acc_row(r, hi) < M_rem) s += acc[tm][tn][r];
            s += __shfl_xor(s, 32, 64);
            const float mean = cnt > 0 ? s / (float)cnt : 0.f;
            float q = 0.f;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (full || wr0 + tm * 32 + acc_row(r, hi) < M_rem) {
                        const float d = acc[tm][tn][r] - mean;
                        q = fmaf(d, d, q);
                    }
            q += __shfl_xor(q, 32, 64);
            if (hi == 0) red[wm * BN + col] = make_float2(mean, q);
        }
        __syncthreads();
        if (wm == 0 && hi == 0) {
            const float na = (float)(M_rem < BM / 2 ? M_rem : BM / 2);
            const float nb = (float)M_rem - na;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = wn * (BN / 2) + tn * 32 + lo;
                const int n = n0 + col;
                const float2 a = red[col], b = red[BN + col];
                float2 o = a;
                if (nb > 0.f) {
                    const float d = b.x - a.x;
                    const float f = nb / (float)M_rem;
                    o.x = a.x + d * f;
                    o.y = a.y + b.y + d * d * na * f;
                }
                if (n < g.N) g.stats[(int64_t)mt * g.N + n] = o;
            }
        }
    }
    if constexpr (EPI == E_BNPART) {
        // per column: this lane's 16*TM rows, the other row half (hi), then the other wave row (LDS);
        // fixed order, so the partials are deterministic
        float2* red = reinterpret_cast<float2*>(&As[0][0]);
        const int ldc = (int)g.ldc;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * (BN / 2) + tn * 32 + lo;
            const int n = n0 + col;
            float s1 = 0.f, s2 = 0.f;
            if (n < g.N) {
                const float sc = g.bsc[n], sh = g.bsh[n];
                const float mu = g.bmu ? g.bmu[n] : 0.f, rs = g.brs ? g.brs[n] : 0.f;
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    const int rb0 = wm * (BM / 2) + tm * 32 + 4 * hi;
                    const float* zp = g.z + (int64_t)(m0 + rb0) * g.ldc + n;
                    float zv[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        zv[r] = (full || rb0 + acc_row(r, 0) < M_rem) ? zp[acc_row(r, 0) * ldc] : 0.f;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const bool in = full || rb0 + acc_row(r, 0) < M_rem;
                        float gm = (in && fmaf(zv[r], sc, sh) > 0.f) ? acc[tm][tn][r] : 0.f;
                        if (g.ep_rate > 0.f)  // (uniform) the consumer read the activation through dropout
                            gm *= drop_mult(g.ep_seed, (uint64_t)(m0 + rb0 + acc_row(r, 0)) * g.N + n, g.ep_rate,
                                            g.ep_inv_keep);
                        s1 += gm;
                        s2 = fmaf(gm, (zv[r] - mu) * rs, s2);
                    }
                }
            }
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (hi == 0) red[wm * BN + col] = make_float2(s1, s2);
        }
        __syncthreads();
        if (wm == 0 && hi == 0) {
            float* out = g.bnpart + (int64_t)mt * 2 * g.N;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = wn * (BN / 2) + tn * 32 + lo;
                const int n = n0 + col;
                const float2 a = red[col], b = red[BN + col];
                if (n < g.N) {
                    out[n] = a.x + b.x;
                    out[g.N + n] = a.y + b.y;
                }
            }
        }
    }
    if constexpr (EPI == E_SHUFFLE) {
        // output pixel offset (a = b = 0 tap) of each tile row: one row per thread through LDS
        // (the loop ended on a barrier) instead of two runtime integer divisions per accumulator
        // row in every thread (~2000 VALU instructions per thread)
        int* orow = reinterpret_cast<int*>(&As[0][0]);
        if (tid < BM) {
            const int m = m0 + tid;
            const int ur = m / g.sW;  // image row over the batch; output row 2 ur, column 2 (m % sW)
            orow[tid] = tid < M_rem ? (4 * ur * g.sW + 2 * (m - ur * g.sW)) * g.sf : -1;
        }
        __syncthreads();
        int obase[TM][16];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int r = 0; r < 16; ++r) obase[tm][r] = orow[wm * (BM / 2) + tm * 32 + acc_row(r, hi)];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * (BN / 2) + tn * 32 + lo;
            if (n >= g.N) continue;
            const int ab = n / g.sf;
            const int co = n - ab * g.sf;
            const int toff = (ab >> 1) * (2 * g.sW * g.sf) + (ab & 1) * g.sf + co;
            const float bias = g.bias ? g.bias[co] : 0.f;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (obase[tm][r] >= 0) g.C[(int64_t)obase[tm][r] + toff] = acc[tm][tn][r] + bias;
        }
    }
    ROWS_STAMP(g, 3);
}

// ------------------------------------------------------------- vectorised wgrad GEMM ----
// X6 (split precision, 128 x 128 tiles): the reduction runs over pixels m, which both operands
// hold m-major, so the bf16 planes are written transposed, [channel][m] with an 80-byte row (32 m +
// 8 pad, conflict-free ds_read_b128 fragments): threads 0-127 stage A, 128-255 B (whole waves), each
// two groups of 4 consecutive m of one channel quad (lane (quad, m-octet) = (u / 4, u % 4)): after an
// in-register 4 x 4 transpose every channel's 4 m go out as one 8-byte store per plane.  As in the
// rows GEMM's X6 route the stages are 32 m deep in ONE LDS buffer (two blocks per CU, two barriers
// per stage), so a stage's matrix work covers the next stage's load latency.
template <int BP, int BQ, int AMODE, bool ADROP, int BMODE, bool BDROP, bool X6 = false>
__global__ __launch_bounds__(256, X6 ? 2 : 1) void gemm_wgrad_vec(WgradArgs g) {
    static_assert(!X6 || (BP == 128 && BQ == 128), "X6 wgrad: 128 x 128 tiles");
    constexpr int KB = X6 ? 32 : BK;                 // m per stage
    constexpr int LDA = BP + 4, LDB = BQ + 4;
    constexpr int TM = BP / 64, TN = BQ / 64;
    constexpr int PQ = BP / 4, QQ = BQ / 4;          // quads per m-row
    constexpr int AR = X6 ? 8 : BK * PQ / 256, BR = X6 ? 8 : BK * QQ / 256;
    constexpr int AS = X6 ? 1 : 256 / PQ, BS = X6 ? 1 : 256 / QQ;  // m-row step between a thread's quads
    constexpr int XW = KB + 8;                       // X6 plane row stride (bf16): 32 m + 8 pad
    constexpr int F32_BYTES = 4 * 2 * BK * (LDA + LDB);
    constexpr int X6_BYTES = 2 * 3 * (BP + BQ) * XW;  // one buffer
    __shared__ __attribute__((aligned(16))) char smem[X6 ? X6_BYTES : F32_BYTES];
    float (*As)[BK * LDA] = reinterpret_cast<float (*)[BK * LDA]>(smem);
    float (*Bs)[BK * LDB] = reinterpret_cast<float (*)[BK * LDB]>(smem + 4 * 2 * BK * LDA);
    unsigned short* Ax = reinterpret_cast<unsigned short*>(smem);  // [plane * BP + p][m]
    unsigned short* Bx = Ax + 3 * BP * XW;                         // [plane * BQ + q][m]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wp = wave >> 1, wq = wave & 1;
    const int lo = lane & 31, hi = lane >> 5;
    const int ntp = (g.P + BP - 1) / BP;
    int tile, slice;  // the (p, q) tiles of an m-slice read the same y / dz rows: one XCD's L2
    xcd_group_order_sx(gridDim.x, gridDim.y, tile, slice);
    const int p0 = (tile % ntp) * BP;
    const int q0 = (tile / ntp) * BQ;
    const int mb = (int)(slice * g.mslice);
    const int me = (int)((mb + g.mslice) < g.M ? (mb + g.mslice) : g.M);
    const bool roleA = !X6 || tid < 128, roleB = !X6 || tid >= 128;
    const int unit = tid & 127;

    const int apq = X6 ? unit >> 2 : tid % PQ, amm = X6 ? 8 * (unit & 3) : tid / PQ;
    const int p = p0 + 4 * apq;
    const bool pv = p < g.P;
    float4 asc = f4(1.f), ash = f4(0.f);
    int poff = p;
    if constexpr (AMODE == W_BNRELU) {
        if (pv) {
            asc = ld4(g.a.sc0 + p);
            ash = ld4(g.a.sh0 + p);
        }
    }
    if constexpr (AMODE == W_UNSHUFFLE) {
        const int ab = p / g.uf;
        const int co = p - ab * g.uf;
        poff = (ab >> 1) * (2 * g.uW * g.uf) + (ab & 1) * g.uf + co;
    }
    const int bqq = X6 ? unit >> 2 : tid % QQ, bmm = X6 ? 8 * (unit & 3) : tid / QQ;
    const int q = q0 + 4 * bqq;
    const bool qv = q < g.Q;
    float4 bsc = f4(1.f), bsh = f4(0.f), bmu = f4(0.f), bp_ = f4(0.f), bq_ = f4(0.f);
    if constexpr (BMODE == W_BNRELU || BMODE == W_BNBWD) {
        if (qv) {
            bsc = ld4(g.b.sc0 + q);
            bsh = ld4(g.b.sh0 + q);
        }
    }
    if constexpr (BMODE == W_BNBWD) {
        if (qv) {
            bmu = ld4(g.bcoef + q);
            bp_ = ld4(g.bcoef + g.Q + q);
            bq_ = ld4(g.bcoef + 2 * g.Q + q);
        }
    }

    float4 ra[AR], rb[BR];
    // W_UNSHUFFLE: pixel m = (image row ur = m / uW over the batch, column uj) of the upsample input;
    // its (0, 0) tap in dU is row 2 ur, column 2 uj.  Tracked incrementally (the stages advance m
    // by BK) instead of two runtime divisions per row and stage.
    int ur[AMODE == W_UNSHUFFLE ? AR : 1], uj[AMODE == W_UNSHUFFLE ? AR : 1];
    if constexpr (AMODE == W_UNSHUFFLE) {
#pragma unroll
        for (int r = 0; r < AR; ++r) {
            const int m = mb + amm + AS * r;
            ur[r] = m / g.uW;
            uj[r] = m - ur[r] * g.uW;
        }
    }
    auto load_stage = [&](int k0) {
#pragma unroll
        for (int r = 0; r < AR; ++r) {
            const int m = k0 + amm + AS * r;
            float4 v = f4(0.f);
            if (roleA && pv && m < me) {
                if constexpr (AMODE == W_UNSHUFFLE) {
                    v = ld4(g.a.src0 + (4 * ur[r] * g.uW + 2 * uj[r]) * g.uf + poff);
                } else {
                    v = ld4(g.a.src0 + (int64_t)m * g.a.c0 + p);
                    if constexpr (AMODE == W_BNRELU) v = bnrelu4(v, asc, ash);
                    if constexpr (ADROP) {
                        const uint64_t i = (uint64_t)m * g.a.C + p;
                        v = mul4(v, drop_mult4(g.a.seed, i, g.a.rate, g.a.inv_keep));
                    }
                }
            }
            ra[r] = v;
        }
#pragma unroll
        for (int r = 0; r < BR; ++r) {
            const int m = k0 + bmm + BS * r;
            float4 v = f4(0.f);
            if (roleB && qv && m < me) {
                v = ld4(g.b.src0 + (int64_t)m * g.b.c0 + q);
                if constexpr (BMODE == W_BNRELU) v = bnrelu4(v, bsc, bsh);
                if constexpr (BMODE == W_BNBWD) {
                    const float4 zz = ld4(g.bz + (int64_t)m * g.b.c0 + q);
                    v.x = fmaf(zz.x, bsc.x, bsh.x) > 0.f ? v.x : 0.f;
                    v.y = fmaf(zz.y, bsc.y, bsh.y) > 0.f ? v.y : 0.f;
                    v.z = fmaf(zz.z, bsc.z, bsh.z) > 0.f ? v.z : 0.f;
                    v.w = fmaf(zz.w, bsc.w, bsh.w) > 0.f ? v.w : 0.f;
                    v.x = bsc.x * (v.x - bp_.x - (zz.x - bmu.x) * bq_.x);
                    v.y = bsc.y * (v.y - bp_.y - (zz.y - bmu.y) * bq_.y);
                    v.z = bsc.z * (v.z - bp_.z - (zz.z - bmu.z) * bq_.z);
                    v.w = bsc.w * (v.w - bp_.w - (zz.w - bmu.w) * bq_.w);
                }
                if constexpr (BDROP) {
                    const uint64_t i = (uint64_t)m * g.b.C + q;
                    v = mul4(v, drop_mult4(g.b.seed, i, g.b.rate, g.b.inv_keep));
                }
            }
            rb[r] = v;
        }
        if constexpr (AMODE == W_UNSHUFFLE) {
#pragma unroll
            for (int r = 0; r < AR; ++r) {
                uj[r] += KB;
                while (uj[r] >= g.uW) {
                    uj[r] -= g.uW;
                    ++ur[r];
                }
            }
        }
    };
    const bool csum_on = g.colpart != nullptr && tile < ntp;  // q-tile 0 blocks sum A's columns
    float4 csum = f4(0.f);
    // X6: 4 consecutive m (rows r = 0..3) of channel c of the thread's quad, split, into the planes
    auto store_t4 = [&](unsigned short* base, int rows, const float4* rv) {
        const float4 cols[4] = {make_float4(rv[0].x, rv[1].x, rv[2].x, rv[3].x),
                                make_float4(rv[0].y, rv[1].y, rv[2].y, rv[3].y),
                                make_float4(rv[0].z, rv[1].z, rv[2].z, rv[3].z),
                                make_float4(rv[0].w, rv[1].w, rv[2].w, rv[3].w)};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const Split4 sp = split4(cols[c]);
            unsigned short* d = base + c * XW;
            *reinterpret_cast<uint2*>(d) = sp.h;
            *reinterpret_cast<uint2*>(d + rows * XW) = sp.m;
            *reinterpret_cast<uint2*>(d + 2 * rows * XW) = sp.l;
        }
    };
    auto store_stage = [&](int buf) {
        if constexpr (X6) {
            if (roleA) {
                store_t4(Ax + 4 * apq * XW + amm, BP, ra);
                store_t4(Ax + 4 * apq * XW + amm + 4, BP, ra + 4);
            } else {
                store_t4(Bx + 4 * bqq * XW + bmm, BQ, rb);
                store_t4(Bx + 4 * bqq * XW + bmm + 4, BQ, rb + 4);
            }
        } else {
#pragma unroll
            for (int r = 0; r < AR; ++r) *reinterpret_cast<float4*>(&As[buf][(amm + AS * r) * LDA + 4 * apq]) = ra[r];
#pragma unroll
            for (int r = 0; r < BR; ++r) *reinterpret_cast<float4*>(&Bs[buf][(bmm + BS * r) * LDB + 4 * bqq]) = rb[r];
        }
        if (csum_on && roleA) {
#pragma unroll
            for (int r = 0; r < AR; ++r) csum = add4(csum, ra[r]);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

    const int nk = (me - mb + KB - 1) / KB;
    if (nk > 0) {
        load_stage(mb);
        store_stage(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_stage(mb + (kt + 1) * KB);
        if constexpr (X6) {
#pragma unroll
            for (int ks = 0; ks < KB / 16; ++ks) {
                bf16x8 bfr[TN][3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        bfr[tn][pl] = *reinterpret_cast<const bf16x8*>(
                            Bx + (pl * BQ + wq * (BQ / 2) + tn * 32 + lo) * XW + ks * 16 + 8 * hi);
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    bf16x8 af[3];
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        af[pl] = *reinterpret_cast<const bf16x8*>(
                            Ax + (pl * BP + wp * (BP / 2) + tm * 32 + lo) * XW + ks * 16 + 8 * hi);
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_x6(af, bfr[tn], acc[tm][tn]);
                }
            }
            __syncthreads();  // one buffer: every wave's fragment reads done before it is rewritten
            if (kt + 1 < nk) {
                store_stage(0);
                __syncthreads();
            }
            continue;
        } else {
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            float av[TM], bv[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) av[tm] = As[buf][(2 * kk + hi) * LDA + wp * (BP / 2) + tm * 32 + lo];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) bv[tn] = Bs[buf][(2 * kk + hi) * LDB + wq * (BQ / 2) + tn * 32 + lo];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[tm], bv[tn], acc[tm][tn], 0, 0, 0);
        }
        }
        if (kt + 1 < nk) store_stage(buf ^ 1);
        __syncthreads();
    }
    if (csum_on) {  // fixed-order sum over the m-rows of each column quad (the loop ended on a barrier)
        float4* T = reinterpret_cast<float4*>(&As[0][0]);
        T[tid] = csum;
        __syncthreads();
        if constexpr (X6) {  // thread u < 128 holds quad u / 4, m-octet u % 4
            if (tid < PQ && p0 + 4 * tid < g.P) {
                float4 t = T[4 * tid];
                for (int j = 1; j < 4; ++j) t = add4(t, T[4 * tid + j]);
                st4(g.colpart + (int64_t)slice * g.P + p0 + 4 * tid, t);
            }
        } else if (tid < PQ && pv) {
            float4 t = T[tid];
            for (int j = 1; j < AS; ++j) t = add4(t, T[j * PQ + tid]);
            st4(g.colpart + (int64_t)slice * g.P + p, t);
        }
    }
    float* slab = g.slab + (int64_t)slice * g.P * g.Q;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int qq = q0 + wq * (BQ / 2) + tn * 32 + lo;
            if (qq >= g.Q) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int pp = p0 + wp * (BP / 2) + tm * 32 + acc_row(r, hi);
                if (pp < g.P) slab[(int64_t)pp * g.Q + qq] = acc[tm][tn][r];
            }
        }
}

// ------------------------------------------------------- image-block data + weight gradient ----
// The image block's pointwise layer is 4 -> C (C = 4G <= 64): its data gradient dy (M x 4) and
// weight gradient dW (4 x C) are two thin reductions over the dz it forms from (da, z), so one
// streaming VALU pass does both (a 4-wide MFMA tile would waste 15/16 of the matrix core): G lanes
// per pixel (one channel quad each), U pixels in flight per lane; dy by xor shuffles over the G
// lanes, dW accumulated per lane over its pixels, then over the lanes / waves of the block into
// one slab per block.
//
// DWF (unet_image_block_bwd_wgrad): the depthwise kernel gradient too.  dy is not stored: it only
// feeds dK[tap][c] = sum_p dy[p, c] x[p + tap offset, c], so once the xor butterfly has given all
// G lanes of a pixel its dy, lane q accumulates taps q and q + G (< 9) against the pixel's
// neighbours in x, loaded beside da / z / y at the top of the iteration (zero outside the image
// and past M).  Slab = [4][C] pointwise | [9][4] depthwise (SW floats).
template <int G, bool DWF = false>
__global__ __launch_bounds__(256) void img_pw_bwd_kernel(const float* __restrict__ da, const float* __restrict__ z,
                                                         int64_t M, const float* __restrict__ P,
                                                         const float* __restrict__ sc, const float* __restrict__ sh,
                                                         const float* __restrict__ coef, const float* __restrict__ y,
                                                         float* __restrict__ dy, float* __restrict__ wpart,
                                                         const float* __restrict__ x = nullptr, int H = 0, int W = 0) {
    main_stream_prio();
    constexpr int C = 4 * G, PPW = 64 / G, U = 4, PB = 4 * U * PPW;
    constexpr int NT = DWF ? (9 + G - 1) / G : 0;  // taps per lane
    constexpr int SW = 4 * C + (DWF ? 36 : 0);   // slab width
    __shared__ float4 red[4][4][G];  // [wave][ci][quad]
    __shared__ float4 rdk[4][DWF ? 9 : 1];  // [wave][tap]
    float4 gacc[NT > 0 ? NT : 1];
#pragma unroll
    for (int i = 0; i < (NT > 0 ? NT : 1); ++i) gacc[i] = f4(0.f);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane % G, ps = lane / G;
    const int c = 4 * q;
    const float4 csc = ld4(sc + c), csh = ld4(sh + c), cmu = ld4(coef + c), cp = ld4(coef + C + c),
                 cq = ld4(coef + 2 * C + c);
    float4 pk[4], wacc[4];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
        pk[ci] = ld4(P + ci * C + c);
        wacc[ci] = f4(0.f);
    }
    for (int64_t base = (int64_t)blockIdx.x * PB; base < M; base += (int64_t)gridDim.x * PB) {
        const int64_t p0 = base + wave * U * PPW + ps;
        float4 ra[U], rz[U], ry[U];
        float4 xn[U][NT > 0 ? NT : 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t m = p0 + u * PPW;
            const bool in = m < M;
            ra[u] = in ? ld4(da + m * C + c) : f4(0.f);
            rz[u] = in ? ld4(z + m * C + c) : f4(0.f);
            ry[u] = in ? ld4(y + m * 4) : f4(0.f);
            if constexpr (DWF) {
                const int mi = in ? (int)m : 0;  // M * C fits int32 (checked on the host)
                const int hw = H * W;
                const int r = mi - (mi / hw) * hw, hh = r / W, ww = r - hh * W;
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    const int t = q + i * G, di = t / 3 - 1, dj = t % 3 - 1;
                    const bool ok = in && t < 9 && hh + di >= 0 && hh + di < H && ww + dj >= 0 && ww + dj < W;
                    xn[u][i] = ok ? ld4(x + (int64_t)(mi + di * W + dj) * 4) : f4(0.f);
                }
            }
        }
        float4 s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float4 zz = rz[u];
            float4 v = ra[u];
            v.x = fmaf(zz.x, csc.x, csh.x) > 0.f ? v.x : 0.f;
            v.y = fmaf(zz.y, csc.y, csh.y) > 0.f ? v.y : 0.f;
            v.z = fmaf(zz.z, csc.z, csh.z) > 0.f ? v.z : 0.f;
            v.w = fmaf(zz.w, csc.w, csh.w) > 0.f ? v.w : 0.f;
            // dz; for a pixel past M it is not 0, but its y is (dW) and its dy is not stored
            v.x = csc.x * (v.x - cp.x - (zz.x - cmu.x) * cq.x);
            v.y = csc.y * (v.y - cp.y - (zz.y - cmu.y) * cq.y);
            v.z = csc.z * (v.z - cp.z - (zz.z - cmu.z) * cq.z);
            v.w = csc.w * (v.w - cp.w - (zz.w - cmu.w) * cq.w);
            s[u].x = v.x * pk[0].x + v.y * pk[0].y + v.z * pk[0].z + v.w * pk[0].w;
            s[u].y = v.x * pk[1].x + v.y * pk[1].y + v.z * pk[1].z + v.w * pk[1].w;
            s[u].z = v.x * pk[2].x + v.y * pk[2].y + v.z * pk[2].z + v.w * pk[2].w;
            s[u].w = v.x * pk[3].x + v.y * pk[3].y + v.z * pk[3].z + v.w * pk[3].w;
            wacc[0] = fma4(v, f4(ry[u].x), wacc[0]);
            wacc[1] = fma4(v, f4(ry[u].y), wacc[1]);
            wacc[2] = fma4(v, f4(ry[u].z), wacc[2]);
            wacc[3] = fma4(v, f4(ry[u].w), wacc[3]);
        }
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                s[u].x += __shfl_xor(s[u].x, off, 64);
                s[u].y += __shfl_xor(s[u].y, off, 64);
                s[u].z += __shfl_xor(s[u].z, off, 64);
                s[u].w += __shfl_xor(s[u].w, off, 64);
            }
        if constexpr (DWF) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int i = 0; i < NT; ++i) gacc[i] = fma4(xn[u][i], s[u], gacc[i]);
        } else if (q == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t m = p0 + u * PPW;
                if (m < M) st4(dy + m * 4, s[u]);
            }
        }
    }
    // dW: lanes of one quad (lane % G) in the wave, then the 4 waves, in a fixed order
#pragma unroll
    for (int off = G; off < 64; off <<= 1)
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            wacc[ci].x += __shfl_xor(wacc[ci].x, off, 64);
            wacc[ci].y += __shfl_xor(wacc[ci].y, off, 64);
            wacc[ci].z += __shfl_xor(wacc[ci].z, off, 64);
            wacc[ci].w += __shfl_xor(wacc[ci].w, off, 64);
        }
    if constexpr (DWF) {
#pragma unroll
        for (int off = G; off < 64; off <<= 1)
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                gacc[i].x += __shfl_xor(gacc[i].x, off, 64);
                gacc[i].y += __shfl_xor(gacc[i].y, off, 64);
                gacc[i].z += __shfl_xor(gacc[i].z, off, 64);
                gacc[i].w += __shfl_xor(gacc[i].w, off, 64);
            }
        if (lane < G) {
#pragma unroll
            for (int i = 0; i < NT; ++i)
                if (lane + i * G < 9) rdk[wave][lane + i * G] = gacc[i];
        }
    }
    if (lane < G) {
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) red[wave][ci][lane] = wacc[ci];
    }
    __syncthreads();
    if (threadIdx.x < 4 * G) {
        const int ci = threadIdx.x / G, qq = threadIdx.x % G;
        const float4 t = add4(add4(red[0][ci][qq], red[1][ci][qq]), add4(red[2][ci][qq], red[3][ci][qq]));
        st4(wpart + (int64_t)blockIdx.x * SW + ci * C + 4 * qq, t);
    }
    if constexpr (DWF) {
        if (threadIdx.x >= 64 && threadIdx.x < 64 + 9) {
            const int t = threadIdx.x - 64;
            const float4 v = add4(add4(rdk[0][t], rdk[1][t]), add4(rdk[2][t], rdk[3][t]));
            st4(wpart + (int64_t)blockIdx.x * SW + 4 * C + 4 * t, v);
        }
    }
    if (blockIdx.x == gridDim.x - 1) {  // zero slabs up to a multiple of 64 (the two-level reduction)
        const int S = gridDim.x, Sp = (S + 63) / 64 * 64;
        for (int i = threadIdx.x; i < (Sp - S) * SW; i += 256) wpart[(int64_t)S * SW + i] = 0.f;
    }
}

// Last level of the image block's weight gradients: T rows of the [4][C] | [9][4] slab summed in
// order (double) and written in the Keras shapes of the 3-channel (wcin) input -- pointwise
// (1, 1, wcin, C), depthwise (3, 3, wcin, 1) -- so no strided copy follows.
__global__ __launch_bounds__(320) void img_wgrad_final_kernel(const float* __restrict__ mid, int T, int C, int wcin,
                                                              float* __restrict__ dpk, float* __restrict__ ddk) {
    const int SW = 4 * C + 36;
    for (int l = threadIdx.x; l < SW; l += blockDim.x) {
        constexpr int TM = 32;  // T <= 32 (2048 slabs / 64): every row's load in flight at once
        float v[TM];
#pragma unroll
        for (int t = 0; t < TM; ++t) v[t] = mid[(int64_t)(t < T ? t : T - 1) * SW + l];
        double a = 0.0;
#pragma unroll
        for (int t = 0; t < TM; ++t)
            if (t < T) a += (double)v[t];
        if (l < 4 * C) {
            const int ci = l / C, co = l - ci * C;
            if (ci < wcin) dpk[ci * C + co] = (float)a;
        } else {
            const int tap = (l - 4 * C) >> 2, ch = (l - 4 * C) & 3;
            if (ch < wcin) ddk[tap * wcin + ch] = (float)a;
        }
    }
}

// ------------------------------------------------------------------------------ launchers ----
bool rows_vec_ok(const RowsArgs& a, int amode) {
    if (a.K % 4 || a.N % 4) return false;
    if (a.sbk * (int64_t)a.K + a.sbn * (int64_t)a.N >= (int64_t(1) << 31)) return false;
    if (amode == A_UNSHUFFLE && a.uf % 4) return false;
    if (amode != A_UNSHUFFLE && a.a.c0 % 4) return false;
    if (a.sbk != 1 && a.sbn != 1) return false;
    return ((uintptr_t)a.a.src0 | (uintptr_t)a.B) % 16 == 0;
}

// Tile configuration of the vectorised rows GEMM: BN columns x BK k per stage (BM = 128).
// Chosen per operand mode from lab timings (tools/lab/gemm_lab.hip) on the U-Net shapes:
// the BatchNorm-backward data gradient forms its A operand per N-tile, so it prefers the
// 256-wide tile when the grid still fills the chip, and BK = 32 otherwise; plain operands
// take BK = 32 from K = 256 on.  Lab build: UNET_ROWS_BN / UNET_ROWS_BK override (tuning only).
struct RowsCfg {
    int bn, bk;
    int bm = 128;
};
RowsCfg rows_cfg(const RowsArgs& a, int amode) {
    const int env_bn = lab_knob("UNET_ROWS_BN", 0);
    if (env_bn > 0) return RowsCfg{env_bn, lab_knob("UNET_ROWS_BK", 16)};
    // grids of 128 x 128 tiles that leave CUs idle (the deep levels at small batch: 2048-8192
    // rows; up to one block per CU) take 64-wide N tiles, twice the blocks (<= 256 rather than
    // < 256 blocks: -0.4 % per step at batch 16 and batch 8, profiles/r5d_step_ab.txt nw_*)
    const bool narrow = lab_knob("UNET_ROWS_NARROW", 1) && a.N > 64 &&
                        cdiv(a.M, 128) * cdiv(a.N, 128) < lab_knob("UNET_ROWS_NARROW_LT", 257);
    if (amode == A_BNBWD) {
        // lab: UNET_BNBWD_BK16 = 1 stages BK = 16 (40 KB of LDS instead of 72 KB at 128 columns:
        // co-residency with the side stream's weight-gradient blocks)
        const int bk = lab_knob("UNET_BNBWD_BK16", 0) ? 16 : 32;
        // under-filled grids (the 16 x 16 level at batch 8): 64-row x 128-column tiles instead of
        // 128 x 64, the same block count with half the N-tiles re-forming each dz tile
        // (tools/lab/gemm_lab.hip LAB_BATCH=8, profiles/r5_lab/r5d_rows_b8.log: 76 -> 65.5 us)
        if (narrow && a.N >= 128 && lab_knob("UNET_BNBWD_BM64", 1)) return RowsCfg{128, 32, 64};
        if (a.N <= 64 || narrow) return RowsCfg{64, bk};
        if (a.N >= 256 && cdiv(a.M, 128) * cdiv(a.N, 256) >= 512) return RowsCfg{256, 16};
        return RowsCfg{128, bk};
    }
    const int bk32_k = lab_knob("UNET_BK32_MIN_K", 256);  // smallest K that takes BK = 32
    if (a.N <= 64) return RowsCfg{64, 16};
    // (the ConvT data gradient keeps BK = 16: BK = 32 runs its kernels 5-20 % faster alone but the
    // step slower beside the side stream, profiles/r5d_step_ab.txt bk_*; lab UNET_UNSHUFFLE_BK32)
    const bool bk32 = a.K >= bk32_k && (amode != A_UNSHUFFLE || lab_knob("UNET_UNSHUFFLE_BK32", 0));
    if (narrow) return RowsCfg{64, bk32 ? 32 : 16};
    return RowsCfg{128, bk32 ? 32 : 16};
}

template <int BN, int BKk, int AMODE, bool DROP, int EPI, bool X6 = false, int BM = 128>
void launch_rows_tile(const RowsArgs& a, hipStream_t st) {
    dim3 grid((unsigned)cdiv(a.M, BM), (unsigned)cdiv(a.N, BN));
    if (X6 || a.sbk == 1) gemm_rows_vec<BM, BN, BKk, AMODE, DROP, EPI, true, X6><<<grid, 256, 0, st>>>(a);
    else gemm_rows_vec<BM, BN, BKk, AMODE, DROP, EPI, false, X6><<<grid, 256, 0, st>>>(a);
}

// Split-precision (bf16x6) rows GEMM: taken when the caller hands pre-split B planes (a.Bx) and
// the k-loop is whole 32-deep stages.  (Round 3's form -- B split in every block, 16-deep stages in
// a double buffer at one block per CU -- was load-latency bound and no faster than fp32 MFMA,
// profiles/r3_x6_rows_ab.jsonl; lab UNET_X6 = 0 turns the route off for A/B runs.)
// Grids of fewer than 256 128 x 128 tiles keep the fp32 route, whose narrow tiles fill the chip (the
// bottleneck's data gradient at batch 16, 32 x 4 tiles: 61 vs 77 us, profiles/r6x_rows_x6.txt), and so
// do outputs of <= 64 columns (enc2_block1's data gradient: 98 us, 110 with 128-column split tiles
// half masked, 110 with 64-column ones, profiles/r6v2_x6_n64.txt).
bool rows_x6(const RowsArgs& a, int amode) {
    return a.Bx != nullptr && a.K % 32 == 0 && a.N > 64 && (amode != A_BNBWD || a.K <= 512) &&
           cdiv(a.M, 128) * cdiv(a.N, 128) >= lab_knob("UNET_X6_MIN_TILES", 256) && lab_knob("UNET_X6", 1) != 0;
}

// Row-tile height of the ConvTranspose data gradient with BatchNorm partials (E_BNPART): 64
// when the 128-row grid holds at most one block per CU (the bottleneck at batch 8: 16 x 16
// blocks of 128 x 64) -- twice the blocks.  The partials are per row tile, so the slab count
// (unet_conv_transpose2x2_bwd_data_bnstats_slabs) follows.  Lab: UNET_CONVT_BM64 = 0 off,
// 2 takes 64 x 128 tiles (the same block count, half the N-tiles).
int convt_bnpart_bm(int64_t M, int N) {
    const int mode = lab_knob("UNET_CONVT_BM64", 1);
    return mode && cdiv(M, 128) * cdiv(N, 64) <= 256 ? 64 : 128;
}

template <int AMODE, bool DROP, int EPI>
int launch_rows(const RowsArgs& a0, hipStream_t st, const char* what) {
    RowsArgs a = a0;
    a.ko = lab_knob("UNET_ROWS_KO", 0);  // 1 no C stores, 2 no dz side copy, 4 no k-loop loads (lab)
    if (rows_vec_ok(a, AMODE)) {
        const RowsCfg c = rows_cfg(a, AMODE);
        if (rows_x6(a, AMODE)) {
            launch_rows_tile<128, 32, AMODE, DROP, EPI, true>(a, st);
            UNET_CHECK_LAUNCH(what);
            return 0;
        }
        if constexpr (AMODE == A_BNBWD && EPI == E_STORE) {
            if (c.bm == 64) {
                launch_rows_tile<128, 32, AMODE, DROP, EPI, false, 64>(a, st);
                UNET_CHECK_LAUNCH(what);
                return 0;
            }
        }
        if constexpr (AMODE == A_UNSHUFFLE && EPI == E_BNPART) {
            if (convt_bnpart_bm(a.M, (int)a.N) == 64) {
                if (lab_knob("UNET_CONVT_BM64", 1) == 2) launch_rows_tile<128, 16, AMODE, DROP, EPI, false, 64>(a, st);
                else if (c.bk == 32) launch_rows_tile<64, 32, AMODE, DROP, EPI, false, 64>(a, st);
                else launch_rows_tile<64, 16, AMODE, DROP, EPI, false, 64>(a, st);
                UNET_CHECK_LAUNCH(what);
                return 0;
            }
        }
        if (c.bn == 64 && c.bk == 16) launch_rows_tile<64, 16, AMODE, DROP, EPI>(a, st);
        else if (c.bn == 64 && c.bk == 32) launch_rows_tile<64, 32, AMODE, DROP, EPI>(a, st);
        else if (c.bn == 128 && c.bk == 32) launch_rows_tile<128, 32, AMODE, DROP, EPI>(a, st);
        else if (c.bn == 256 && c.bk == 16) launch_rows_tile<256, 16, AMODE, DROP, EPI>(a, st);
        else launch_rows_tile<128, 16, AMODE, DROP, EPI>(a, st);
        UNET_CHECK_LAUNCH(what);
        return 0;
    }
    if constexpr (AMODE == A_BNBWD || EPI == E_BNPART) {  // vectorised kernel only
        UNET_CHECK_ARG(false, "%s: needs channel counts divisible by 4 and 16-B aligned operands", what);
    } else {
        const unsigned gm = (unsigned)cdiv(a.M, 128);
        if (a.N <= 64) {
            dim3 grid(gm, (unsigned)cdiv(a.N, 64));
            gemm_rows_kernel<128, 64, AMODE, DROP, EPI><<<grid, 256, 0, st>>>(a);
        } else {
            dim3 grid(gm, (unsigned)cdiv(a.N, 128));
            gemm_rows_kernel<128, 128, AMODE, DROP, EPI><<<grid, 256, 0, st>>>(a);
        }
        UNET_CHECK_LAUNCH(what);
    }
    return 0;
}

struct WgradPlan {
    int bp, bq, tiles, S;
    int64_t mslice;
};
WgradPlan wgrad_plan(int64_t M, int P, int Q) {
    WgradPlan w;
    w.bp = P > 64 ? 128 : 64;
    w.bq = Q > 64 ? 128 : 64;
    w.tiles = (int)(cdiv(P, w.bp) * cdiv(Q, w.bq));
    int target = lab_knob("UNET_WGRAD_BLOCKS", 1024);  // ~4 blocks per CU
    if (target < 1) target = 1024;
    int64_t want = cdiv(target, w.tiles);
    int64_t maxs = M / lab_knob("UNET_WGRAD_MINROWS", 512);  // >= 32 k-steps per block: fewer, cheaper slabs
    if (maxs < 1) maxs = 1;
    int64_t S = want < maxs ? want : maxs;
    if (S < 1) S = 1;
    w.mslice = cdiv(cdiv(M, S), BK) * BK;
    w.S = (int)cdiv(M, w.mslice);
    return w;
}

// Split-precision weight gradients (both operands split as they are staged, 128 x 128 tiles): lab
// only.  Slower than fp32 MFMA on every train-step shape (0.71-0.99x isolated, step 10.80 vs 9.85 ms,
// profiles/r6w_wgrad_x6_ab.txt): both operands pay the transpose + split VALU inside the 16-stage
// slices of the split-K grid, with no pre-split operand to lean on.
bool wgrad_x6() { return lab_knob("UNET_WGRAD_X6", 0) != 0; }

template <int AMODE, bool ADROP, int BMODE, bool BDROP>
void launch_wgrad_t(const WgradArgs& a, const WgradPlan& w, hipStream_t st) {
    dim3 grid((unsigned)w.tiles, (unsigned)w.S);
    const unsigned pad = (unsigned)lab_knob("UNET_WGRAD_LDSPAD", 0);  // lab: dynamic LDS pad (fewer blocks per CU)
    const bool vec = a.P % 4 == 0 && a.Q % 4 == 0 && (AMODE != W_UNSHUFFLE || a.uf % 4 == 0) &&
                     (AMODE == W_UNSHUFFLE || a.a.c0 % 4 == 0) && a.b.c0 % 4 == 0 &&
                     ((uintptr_t)a.a.src0 | (uintptr_t)a.b.src0) % 16 == 0;
    if (vec || BMODE == W_BNBWD) {
        if (w.bp == 128 && w.bq == 128 && a.x6 && wgrad_x6()) {
            gemm_wgrad_vec<128, 128, AMODE, ADROP, BMODE, BDROP, true><<<grid, 256, pad, st>>>(a);
            return;
        }
        if (w.bp == 128 && w.bq == 128)
            gemm_wgrad_vec<128, 128, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
        else if (w.bp == 128)
            gemm_wgrad_vec<128, 64, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
        else if (w.bq == 128)
            gemm_wgrad_vec<64, 128, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
        else
            gemm_wgrad_vec<64, 64, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
        return;
    }
    if constexpr (BMODE == W_BNBWD) return;  // (unreachable: the vectorised kernel above)
    else if (w.bp == 128 && w.bq == 128)
        gemm_wgrad_kernel<128, 128, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
    else if (w.bp == 128)
        gemm_wgrad_kernel<128, 64, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
    else if (w.bq == 128)
        gemm_wgrad_kernel<64, 128, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
    else
        gemm_wgrad_kernel<64, 64, AMODE, ADROP, BMODE, BDROP><<<grid, 256, pad, st>>>(a);
}

// out[P][Q] (row stride ldo) = sum_m A(m, p) B(m, q)
int run_wgrad(WgradArgs a, int amode, int bmode, float* out, void* ws, size_t ws_bytes, hipStream_t st,
              const char* what) {
    WgradPlan w = wgrad_plan(a.M, a.P, a.Q);
    const size_t need = (size_t)w.S * a.P * a.Q * sizeof(float);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "%s: workspace %zu < %zu", what, ws_bytes, need);
    a.mslice = w.mslice;
    a.slab = static_cast<float*>(ws);
    a.x6 = true;
    const bool ad = a.a.rate > 0.f, bd = a.b.rate > 0.f;
    if (amode == W_PLAIN && bmode == W_PLAIN) {
        launch_wgrad_t<W_PLAIN, false, W_PLAIN, false>(a, w, st);
    } else if (amode == W_UNSHUFFLE && bmode == W_BNRELU) {
        if (bd)
            launch_wgrad_t<W_UNSHUFFLE, false, W_BNRELU, true>(a, w, st);
        else
            launch_wgrad_t<W_UNSHUFFLE, false, W_BNRELU, false>(a, w, st);
    } else if (amode == W_UNSHUFFLE && bmode == W_PLAIN) {
        if (bd)
            launch_wgrad_t<W_UNSHUFFLE, false, W_PLAIN, true>(a, w, st);
        else
            launch_wgrad_t<W_UNSHUFFLE, false, W_PLAIN, false>(a, w, st);
    } else if (amode == W_BNRELU && bmode == W_PLAIN) {
        if (ad)
            launch_wgrad_t<W_BNRELU, true, W_PLAIN, false>(a, w, st);
        else
            launch_wgrad_t<W_BNRELU, false, W_PLAIN, false>(a, w, st);
    } else {
        UNET_CHECK_ARG(false, "%s: unsupported wgrad operand modes %d/%d", what, amode, bmode);
    }
    UNET_CHECK_LAUNCH(what);
    return reduce_slabs(a.slab, w.S, (int64_t)a.P * a.Q, out, (int64_t)a.P * a.Q, (int64_t)a.P * a.Q, st);
}

size_t wgrad_workspace(int64_t M, int P, int Q) {
    WgradPlan w = wgrad_plan(M, P, Q);
    return align_up((size_t)w.S * P * Q * sizeof(float), 256);
}

DView plain_view(const float* p, int c) {
    unet_view v{};
    v.mode = UNET_VIEW_PLAIN;
    v.c0 = c;
    v.src0 = p;
    return make_dview(v);
}

bool fits_i32(int64_t a, int64_t b) { return a * b < (int64_t(1) << 31); }

}  // namespace
}  // namespace unet

using namespace unet;

// ------------------------------------------------------------------- pointwise conv ----
extern "C" size_t unet_bn_partials_size(int64_t m, int c) {
    if (m <= 0 || c <= 0) return 0;
    return bn_partials_bytes(m, c);  // partials + the finalize's chunk scratch (bn.hip)
}

namespace {
int pw_fwd(const float* y, int64_t m, int cin, int cout, const float* pw_kernel, const unsigned short* pw_kernel_x3,
           float* z, float* bn_partials, unet_stream_t stream) {
    UNET_CHECK_ARG(y && pw_kernel && z, "unet_pointwise_fwd: null pointer");
    UNET_CHECK_ARG(m > 0 && cin > 0 && cout > 0, "unet_pointwise_fwd: bad sizes");
    UNET_CHECK_ARG(fits_i32(m, cin) && fits_i32(m, cout), "unet_pointwise_fwd: tensor too large");
    RowsArgs a{};
    a.a = plain_view(y, cin);
    a.M = m;
    a.K = cin;
    a.B = pw_kernel;
    a.Bx = pw_kernel_x3;  // [3][cout][cin]: k = ci contiguous
    a.sbk = cout;
    a.sbn = 1;
    a.N = cout;
    a.C = z;
    a.ldc = cout;
    a.stats = reinterpret_cast<float2*>(bn_partials);
    hipStream_t st = as_stream(stream);
    if (bn_partials) return launch_rows<A_PLAIN, false, E_STATS>(a, st, "unet_pointwise_fwd");
    return launch_rows<A_PLAIN, false, E_STORE>(a, st, "unet_pointwise_fwd");
}
}  // namespace

extern "C" int unet_pointwise_fwd(const float* y, int64_t m, int cin, int cout, const float* pw_kernel, float* z,
                                  float* bn_partials, unet_stream_t stream) {
    return pw_fwd(y, m, cin, cout, pw_kernel, nullptr, z, bn_partials, stream);
}
extern "C" int unet_pointwise_fwd_x3(const float* y, int64_t m, int cin, int cout, const float* pw_kernel,
                                     const unsigned short* pw_kernel_x3, float* z, float* bn_partials,
                                     unet_stream_t stream) {
    UNET_CHECK_ARG(pw_kernel_x3 && (uintptr_t)pw_kernel_x3 % 16 == 0,
                   "unet_pointwise_fwd_x3: pw_kernel_x3 must be a 16-B aligned plane set");
    return pw_fwd(y, m, cin, cout, pw_kernel, pw_kernel_x3, z, bn_partials, stream);
}

extern "C" int unet_pointwise_bwd_data(const float* dz, int64_t m, int cin, int cout, const float* pw_kernel,
                                       float* dy, unet_stream_t stream) {
    UNET_CHECK_ARG(dz && pw_kernel && dy, "unet_pointwise_bwd_data: null pointer");
    UNET_CHECK_ARG(m > 0 && cin > 0 && cout > 0, "unet_pointwise_bwd_data: bad sizes");
    UNET_CHECK_ARG(fits_i32(m, cin) && fits_i32(m, cout), "unet_pointwise_bwd_data: tensor too large");
    RowsArgs a{};
    a.a = plain_view(dz, cout);
    a.M = m;
    a.K = cout;
    a.B = pw_kernel;  // B(k = co, n = ci) = k[ci][co]
    a.sbk = 1;
    a.sbn = cout;
    a.N = cin;
    a.C = dy;
    a.ldc = cin;
    return launch_rows<A_PLAIN, false, E_STORE>(a, as_stream(stream), "unet_pointwise_bwd_data");
}

namespace {
// dz of a BatchNorm + ReLU (+ dropout) block output from (da, z) and coef = (mu, p, q), exactly as
// the A_BNBWD operand load forms it: one streaming pass (float4 per thread-iteration).
template <bool DROP>
__global__ __launch_bounds__(256) void bn_bwd_dz_kernel(const float* __restrict__ da, const float* __restrict__ z,
                                                        int64_t M, int C, const float* __restrict__ sc,
                                                        const float* __restrict__ sh, const float* __restrict__ coef,
                                                        float rate, float inv_keep, uint64_t seed,
                                                        float* __restrict__ dz) {
    const int CQ = C / 4;
    const int total = (int)(M * CQ);  // < 2^29 (the caller checks M * C < 2^31): 32-bit index math
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
        const int c = (idx % CQ) * 4;
        const int o = idx * 4;  // = m * C + c
        float4 v = ld4(da + o);
        const float4 zz = ld4(z + o), csc = ld4(sc + c), csh = ld4(sh + c);
        const float4 cmu = ld4(coef + c), cp = ld4(coef + C + c), cq = ld4(coef + 2 * C + c);
        if constexpr (DROP) v = mul4(v, drop_mult4(seed, (uint64_t)o, rate, inv_keep));
        v.x = fmaf(zz.x, csc.x, csh.x) > 0.f ? v.x : 0.f;
        v.y = fmaf(zz.y, csc.y, csh.y) > 0.f ? v.y : 0.f;
        v.z = fmaf(zz.z, csc.z, csh.z) > 0.f ? v.z : 0.f;
        v.w = fmaf(zz.w, csc.w, csh.w) > 0.f ? v.w : 0.f;
        v.x = csc.x * (v.x - cp.x - (zz.x - cmu.x) * cq.x);
        v.y = csc.y * (v.y - cp.y - (zz.y - cmu.y) * cq.y);
        v.z = csc.z * (v.z - cp.z - (zz.z - cmu.z) * cq.z);
        v.w = csc.w * (v.w - cp.w - (zz.w - cmu.w) * cq.w);
        st4(dz + o, v);
    }
}
}  // namespace

namespace {
int pw_bwd_data_bnrelu(const float* da, const float* z, int64_t m, int cin, int cout, const float* pw_kernel,
                       const unsigned short* pw_kernel_x3, const float* scale, const float* shift, const float* coef,
                       float drop_rate, uint64_t drop_seed, float* dy, float* dz, unet_stream_t stream) {
    UNET_CHECK_ARG(da && z && pw_kernel && scale && shift && coef && dy, "unet_pointwise_bwd_data_bnrelu: null pointer");
    UNET_CHECK_ARG(m > 0 && cin > 0 && cout > 0, "unet_pointwise_bwd_data_bnrelu: bad sizes");
    UNET_CHECK_ARG(fits_i32(m, cin) && fits_i32(m, cout), "unet_pointwise_bwd_data_bnrelu: tensor too large");
    UNET_CHECK_ARG(drop_rate >= 0.f && drop_rate < 1.f, "unet_pointwise_bwd_data_bnrelu: bad drop_rate");
    UNET_CHECK_ARG(((uintptr_t)z | (uintptr_t)coef | (uintptr_t)scale | (uintptr_t)shift | (uintptr_t)dz) % 16 == 0,
                   "unet_pointwise_bwd_data_bnrelu: operands must be 16-B aligned");
    RowsArgs a{};
    a.a = plain_view(da, cout);
    a.a.sc0 = scale;
    a.a.sh0 = shift;
    a.a.rate = drop_rate;
    a.a.inv_keep = drop_rate > 0.f ? 1.0f / (1.0f - drop_rate) : 1.0f;
    a.a.seed = drop_seed;
    a.z = z;
    a.coef = coef;
    a.side = dz;
    a.M = m;
    a.K = cout;
    a.B = pw_kernel;  // B(k = co, n = ci) = k[ci][co]
    a.Bx = pw_kernel_x3;
    a.sbk = 1;
    a.sbn = cout;
    a.N = cin;
    a.C = dy;
    a.ldc = cin;
    hipStream_t st = as_stream(stream);
    // The bottleneck-adjacent data gradients (1024 channels on either side: 4+ N-tiles of 256 each
    // re-forming the same dz tile from (da, z), or 1024-deep k-loops of the BN-backward operand
    // load) form dz once in a streaming pass (~6 TB/s) and run the plain GEMM on it: 12-24 us
    // faster per launch (tools/bench_dgrad.py, profiles/r2h_dgrad_split.log); narrower shapes
    // measured equal or slower that way and keep the fused operand load.
    if (dz && (cin >= 1024 || cout >= 1024) && cout % 4 == 0 && rows_vec_ok(a, A_BNBWD)) {
        const int64_t work = m * (cout / 4);
        const unsigned grid = (unsigned)(work / 256 < 4096 ? cdiv(work, 256) : 4096);
        if (drop_rate > 0.f)
            bn_bwd_dz_kernel<true><<<grid, 256, 0, st>>>(da, z, m, cout, scale, shift, coef, drop_rate, a.a.inv_keep,
                                                         drop_seed, dz);
        else
            bn_bwd_dz_kernel<false><<<grid, 256, 0, st>>>(da, z, m, cout, scale, shift, coef, 0.f, 1.f, 0, dz);
        UNET_CHECK_LAUNCH("unet_pointwise_bwd_data_bnrelu(dz)");
        RowsArgs p{};
        p.a = plain_view(dz, cout);
        p.M = m;
        p.K = cout;
        p.B = pw_kernel;
        p.Bx = pw_kernel_x3;
        p.sbk = 1;
        p.sbn = cout;
        p.N = cin;
        p.C = dy;
        p.ldc = cin;
        return launch_rows<A_PLAIN, false, E_STORE>(p, st, "unet_pointwise_bwd_data_bnrelu");
    }
    if (drop_rate > 0.f)
        return launch_rows<A_BNBWD, true, E_STORE>(a, st, "unet_pointwise_bwd_data_bnrelu");
    return launch_rows<A_BNBWD, false, E_STORE>(a, st, "unet_pointwise_bwd_data_bnrelu");
}
}  // namespace

extern "C" int unet_pointwise_bwd_data_bnrelu(const float* da, const float* z, int64_t m, int cin, int cout,
                                              const float* pw_kernel, const float* scale, const float* shift,
                                              const float* coef, float drop_rate, uint64_t drop_seed, float* dy,
                                              float* dz, unet_stream_t stream) {
    return pw_bwd_data_bnrelu(da, z, m, cin, cout, pw_kernel, nullptr, scale, shift, coef, drop_rate, drop_seed, dy,
                              dz, stream);
}

extern "C" int unet_pointwise_bwd_data_bnrelu_x3(const float* da, const float* z, int64_t m, int cin, int cout,
                                                 const float* pw_kernel, const unsigned short* pw_kernel_x3,
                                                 const float* scale, const float* shift, const float* coef,
                                                 float drop_rate, uint64_t drop_seed, float* dy, float* dz,
                                                 unet_stream_t stream) {
    UNET_CHECK_ARG(pw_kernel_x3 && (uintptr_t)pw_kernel_x3 % 16 == 0,
                   "unet_pointwise_bwd_data_bnrelu_x3: pw_kernel_x3 must be a 16-B aligned plane set");
    return pw_bwd_data_bnrelu(da, z, m, cin, cout, pw_kernel, pw_kernel_x3, scale, shift, coef, drop_rate, drop_seed,
                              dy, dz, stream);
}

namespace {
int img_pw_slabs(int64_t m, int cout) {
    const int64_t pb = 16 * (64 / (cout / 4));  // pixels per block iteration
    const int64_t g = cdiv(m, pb);
    return (int)(g < 2048 ? g : 2048);
}
}  // namespace

extern "C" size_t unet_pointwise_bwd_data_bnrelu_wgrad_workspace(int64_t m, int cin, int cout) {
    if (m <= 0 || cin != 4 || (cout != 32 && cout != 64)) return 0;
    const int64_t sp = cdiv(img_pw_slabs(m, cout), 64) * 64;  // slabs, padded to 64 groups of sp/64
    return align_up((size_t)sp * 4 * cout * sizeof(float), 256) +
           align_up((size_t)(sp / 64) * 4 * cout * sizeof(float), 256);
}

extern "C" int unet_pointwise_bwd_data_bnrelu_wgrad(const float* da, const float* z, int64_t m, int cin, int cout,
                                                    const float* pw_kernel, const float* scale, const float* shift,
                                                    const float* coef, const float* y, float* dy, float* d_pw_kernel,
                                                    void* ws, size_t ws_bytes, unet_stream_t stream) {
    UNET_CHECK_ARG(da && z && pw_kernel && scale && shift && coef && y && dy && d_pw_kernel,
                   "unet_pointwise_bwd_data_bnrelu_wgrad: null pointer");
    UNET_CHECK_ARG(m > 0 && cin == 4 && (cout == 32 || cout == 64),
                   "unet_pointwise_bwd_data_bnrelu_wgrad: needs cin == 4 and cout 32 or 64");
    UNET_CHECK_ARG(fits_i32(m, cout), "unet_pointwise_bwd_data_bnrelu_wgrad: tensor too large");
    UNET_CHECK_ARG(((uintptr_t)da | (uintptr_t)z | (uintptr_t)coef | (uintptr_t)scale | (uintptr_t)shift |
                    (uintptr_t)y | (uintptr_t)dy | (uintptr_t)pw_kernel | (uintptr_t)ws) % 16 == 0,
                   "unet_pointwise_bwd_data_bnrelu_wgrad: operands must be 16-B aligned");
    const size_t need = unet_pointwise_bwd_data_bnrelu_wgrad_workspace(m, cin, cout);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_pointwise_bwd_data_bnrelu_wgrad: workspace %zu < %zu", ws_bytes,
                   need);
    hipStream_t st = as_stream(stream);
    const int S = img_pw_slabs(m, cout);
    float* part = static_cast<float*>(ws);
    if (cout == 64)
        img_pw_bwd_kernel<16><<<S, 256, 0, st>>>(da, z, m, pw_kernel, scale, shift, coef, y, dy, part);
    else
        img_pw_bwd_kernel<8><<<S, 256, 0, st>>>(da, z, m, pw_kernel, scale, shift, coef, y, dy, part);
    UNET_CHECK_LAUNCH("unet_pointwise_bwd_data_bnrelu_wgrad");
    // two fixed-order levels (up to 2048 slabs of 4*cout floats; one level would run on a few blocks):
    // 64 groups of T = sp/64 slabs -> T slabs, then T -> 1
    const int64_t L = (int64_t)4 * cout, sp = cdiv(S, 64) * 64, T = sp / 64;
    float* mid = reinterpret_cast<float*>(static_cast<char*>(ws) + align_up((size_t)sp * L * sizeof(float), 256));
    int rc = reduce_slabs(part, 64, T * L, mid, T * L, T * L, st);
    if (rc) return rc;
    return reduce_slabs(mid, (int)T, L, d_pw_kernel, L, L, st);
}

extern "C" size_t unet_image_block_bwd_wgrad_workspace(int n, int h, int w, int cout) {
    const int64_t m = (int64_t)n * h * w;
    if (m <= 0 || (cout != 32 && cout != 64)) return 0;
    const int64_t sp = cdiv(img_pw_slabs(m, cout), 64) * 64, L = 4 * cout + 36;
    return align_up((size_t)sp * L * sizeof(float), 256) + align_up((size_t)(sp / 64) * L * sizeof(float), 256);
}

extern "C" int unet_image_block_bwd_wgrad(const float* x, int n, int h, int w, int wcin, int cout,
                                          const float* pw_kernel, const float* scale, const float* shift,
                                          const float* coef, const float* da, const float* z, const float* y,
                                          float* d_dw_kernel, float* d_pw_kernel, void* ws, size_t ws_bytes,
                                          unet_stream_t stream) {
    UNET_CHECK_ARG(x && pw_kernel && scale && shift && coef && da && z && y && d_dw_kernel && d_pw_kernel,
                   "unet_image_block_bwd_wgrad: null pointer");
    UNET_CHECK_ARG(n > 0 && h > 0 && w > 0 && wcin >= 1 && wcin <= 4 && (cout == 32 || cout == 64),
                   "unet_image_block_bwd_wgrad: needs n, h, w > 0, 1 <= wcin <= 4 and cout 32 or 64");
    const int64_t m = (int64_t)n * h * w;
    UNET_CHECK_ARG(fits_i32(m, cout), "unet_image_block_bwd_wgrad: tensor too large");
    UNET_CHECK_ARG(((uintptr_t)x | (uintptr_t)da | (uintptr_t)z | (uintptr_t)coef | (uintptr_t)scale |
                    (uintptr_t)shift | (uintptr_t)y | (uintptr_t)pw_kernel | (uintptr_t)ws) % 16 == 0,
                   "unet_image_block_bwd_wgrad: operands must be 16-B aligned");
    const size_t need = unet_image_block_bwd_wgrad_workspace(n, h, w, cout);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_image_block_bwd_wgrad: workspace %zu < %zu", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    const int S = img_pw_slabs(m, cout);
    const int64_t L = (int64_t)4 * cout + 36, sp = cdiv(S, 64) * 64, T = sp / 64;
    // checked before any launch (img_wgrad_final_kernel holds <= 32 slab rows in registers)
    UNET_CHECK_ARG(T <= 32, "unet_image_block_bwd_wgrad: %d slab rows > 32", (int)T);
    float* part = static_cast<float*>(ws);
    if (cout == 64)
        img_pw_bwd_kernel<16, true><<<S, 256, 0, st>>>(da, z, m, pw_kernel, scale, shift, coef, y, nullptr, part, x,
                                                       h, w);
    else
        img_pw_bwd_kernel<8, true><<<S, 256, 0, st>>>(da, z, m, pw_kernel, scale, shift, coef, y, nullptr, part, x,
                                                      h, w);
    UNET_CHECK_LAUNCH("unet_image_block_bwd_wgrad");
    float* mid = reinterpret_cast<float*>(static_cast<char*>(ws) + align_up((size_t)sp * L * sizeof(float), 256));
    int rc = reduce_slabs(part, 64, T * L, mid, T * L, T * L, st);
    if (rc) return rc;
    img_wgrad_final_kernel<<<1, 320, 0, st>>>(mid, (int)T, cout, wcin, d_pw_kernel, d_dw_kernel);
    UNET_CHECK_LAUNCH("unet_image_block_bwd_wgrad(final)");
    return 0;
}

extern "C" size_t unet_pointwise_bwd_filter_workspace(int64_t m, int cin, int cout) {
    if (m <= 0 || cin <= 0 || cout <= 0) return 0;
    return wgrad_workspace(m, cin, cout);
}

extern "C" int unet_pointwise_bwd_filter(const float* y, const float* dz, int64_t m, int cin, int cout,
                                         float* d_pw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream) {
    UNET_CHECK_ARG(y && dz && d_pw_kernel, "unet_pointwise_bwd_filter: null pointer");
    UNET_CHECK_ARG(m > 0 && cin > 0 && cout > 0, "unet_pointwise_bwd_filter: bad sizes");
    WgradArgs a{};
    a.a = plain_view(y, cin);
    a.P = cin;
    a.b = plain_view(dz, cout);
    a.Q = cout;
    a.M = m;
    return run_wgrad(a, W_PLAIN, W_PLAIN, d_pw_kernel, ws, ws_bytes, as_stream(stream), "unet_pointwise_bwd_filter");
}

// ------------------------------------------------------------ transposed conv 2x2/2 ----
namespace {
int convt_fwd(const unet_view* x, int n, int h, int w, int cout, const float* kernel, const unsigned short* kernel_x3,
              const float* bias, float* out, unet_stream_t stream) {
    if (check_view(x, "unet_conv_transpose2x2_fwd")) return -1;
    UNET_CHECK_ARG(x->mode == UNET_VIEW_PLAIN || x->mode == UNET_VIEW_BNRELU,
                   "unet_conv_transpose2x2_fwd: input view must be PLAIN or BNRELU");
    UNET_CHECK_ARG(kernel && out && n > 0 && h > 0 && w > 0 && cout > 0, "unet_conv_transpose2x2_fwd: bad args");
    const int cin = x->c0;
    const int64_t M = (int64_t)n * h * w;
    UNET_CHECK_ARG(fits_i32(M, cin) && fits_i32(4 * M, cout), "unet_conv_transpose2x2_fwd: tensor too large");
    RowsArgs a{};
    a.a = make_dview(*x);
    a.M = M;
    a.K = cin;
    a.B = kernel;  // B(k = ci, n = (a, b, co)) = k[(a*2+b)*cout + co][ci]
    a.Bx = kernel_x3;
    a.sbk = 1;
    a.sbn = cin;
    a.N = 4 * cout;
    a.C = out;
    a.bias = bias;
    a.sH = h;
    a.sW = w;
    a.sf = cout;
    hipStream_t st = as_stream(stream);
    const bool drop = x->drop_rate > 0.f;
    if (x->mode == UNET_VIEW_PLAIN) {
        if (drop) return launch_rows<A_PLAIN, true, E_SHUFFLE>(a, st, "unet_conv_transpose2x2_fwd");
        return launch_rows<A_PLAIN, false, E_SHUFFLE>(a, st, "unet_conv_transpose2x2_fwd");
    }
    if (drop) return launch_rows<A_BNRELU, true, E_SHUFFLE>(a, st, "unet_conv_transpose2x2_fwd");
    return launch_rows<A_BNRELU, false, E_SHUFFLE>(a, st, "unet_conv_transpose2x2_fwd");
}
}  // namespace

extern "C" int unet_conv_transpose2x2_fwd(const unet_view* x, int n, int h, int w, int cout, const float* kernel,
                                          const float* bias, float* out, unet_stream_t stream) {
    return convt_fwd(x, n, h, w, cout, kernel, nullptr, bias, out, stream);
}
extern "C" int unet_conv_transpose2x2_fwd_x3(const unet_view* x, int n, int h, int w, int cout, const float* kernel,
                                             const unsigned short* kernel_x3, const float* bias, float* out,
                                             unet_stream_t stream) {
    UNET_CHECK_ARG(kernel_x3 && (uintptr_t)kernel_x3 % 16 == 0,
                   "unet_conv_transpose2x2_fwd_x3: kernel_x3 must be a 16-B aligned plane set");
    return convt_fwd(x, n, h, w, cout, kernel, kernel_x3, bias, out, stream);
}

namespace {
bool convt_fused_bias() {  // lab build UNET_CONVT_FUSED_BIAS=0: separate colsum pass (A/B switch)
    return lab_knob("UNET_CONVT_FUSED_BIAS", 1) != 0;
}
}  // namespace

extern "C" size_t unet_conv_transpose2x2_bwd_workspace(int n, int h, int w, int cin, int cout) {
    if (n <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return 0;
    const int64_t M = (int64_t)n * h * w;
    const WgradPlan wp = wgrad_plan(M, 4 * cout, cin);
    size_t a = wgrad_workspace(M, 4 * cout, cin) + align_up((size_t)wp.S * 4 * cout * sizeof(float), 256);
    size_t b = colsum_workspace(4 * M, cout);
    return a > b ? a : b;
}

extern "C" int unet_conv_transpose2x2_bwd(const unet_view* x, int n, int h, int w, int cout, const float* kernel,
                                          const float* dout, float* dx, float* dkernel, float* dbias, void* ws,
                                          size_t ws_bytes, unet_stream_t stream) {
    if (check_view(x, "unet_conv_transpose2x2_bwd")) return -1;
    UNET_CHECK_ARG(x->mode == UNET_VIEW_PLAIN || x->mode == UNET_VIEW_BNRELU,
                   "unet_conv_transpose2x2_bwd: input view must be PLAIN or BNRELU");
    UNET_CHECK_ARG(kernel && dout && n > 0 && h > 0 && w > 0 && cout > 0, "unet_conv_transpose2x2_bwd: bad args");
    UNET_CHECK_ARG((dkernel == nullptr) == (dbias == nullptr) && (dx || dkernel),
                   "unet_conv_transpose2x2_bwd: dkernel and dbias go together; nothing to compute");
    const int cin = x->c0;
    const int64_t M = (int64_t)n * h * w;
    UNET_CHECK_ARG(fits_i32(M, cin) && fits_i32(4 * M, cout), "unet_conv_transpose2x2_bwd: tensor too large");
    hipStream_t st = as_stream(stream);
    const size_t need = unet_conv_transpose2x2_bwd_workspace(n, h, w, cin, cout);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_conv_transpose2x2_bwd: workspace %zu < %zu", ws_bytes, need);
    // data gradient w.r.t. the view output: dx[m, ci] = sum_{(a,b,co)} dU'[m, (a,b,co)] k[(a,b,co)][ci]
    if (dx) {
        RowsArgs a{};
        a.a = plain_view(dout, cout);
        a.M = M;
        a.K = 4 * cout;
        a.uH = h;
        a.uW = w;
        a.uf = cout;
        a.B = kernel;
        a.sbk = cin;
        a.sbn = 1;
        a.N = cin;
        a.C = dx;
        a.ldc = cin;
        int rc = launch_rows<A_UNSHUFFLE, false, E_STORE>(a, st, "unet_conv_transpose2x2_bwd(data)");
        if (rc) return rc;
    }
    if (!dkernel) return 0;  // data gradient only
    // kernel gradient: dk[(a,b,co)][ci] = sum_m dU'[m, (a,b,co)] x[m, ci]
    WgradArgs wa{};
    wa.a = plain_view(dout, cout);
    wa.P = 4 * cout;
    wa.uH = h;
    wa.uW = w;
    wa.uf = cout;
    wa.b = make_dview(*x);
    wa.Q = cin;
    wa.M = M;
    // bias gradient: the q-tile-0 blocks of the kernel-gradient GEMM also sum dU' over their m slice
    // ([S][4][cout] after the slabs), so dU' is read once; = one fixed-order reduction of 4S rows
    const WgradPlan wp = wgrad_plan(M, 4 * cout, cin);
    const size_t slab_bytes = align_up((size_t)wp.S * 4 * cout * cin * sizeof(float), 256);
    const bool fuse_bias = convt_fused_bias() && cin % 4 == 0 && cout % 4 == 0 &&
                           ((uintptr_t)dout | (uintptr_t)x->src0) % 16 == 0 &&
                           ws_bytes >= slab_bytes + (size_t)wp.S * 4 * cout * sizeof(float);
    if (fuse_bias) wa.colpart = reinterpret_cast<float*>(static_cast<char*>(ws) + slab_bytes);
    int rc = run_wgrad(wa, W_UNSHUFFLE, x->mode == UNET_VIEW_BNRELU ? W_BNRELU : W_PLAIN, dkernel, ws, ws_bytes, st,
                       "unet_conv_transpose2x2_bwd(filter)");
    if (rc) return rc;
    if (fuse_bias) return reduce_slabs(wa.colpart, 4 * wp.S, cout, dbias, cout, cout, st);
    return colsum(dout, 4 * M, cout, dbias, ws, ws_bytes, st);
}

extern "C" int unet_conv_transpose2x2_bwd_data_bnstats_slabs(const unet_view* x, int n, int h, int w, int cout) {
    if (!x || x->mode != UNET_VIEW_BNRELU || !(x->drop_rate >= 0.f && x->drop_rate < 1.f) || n <= 0 || h <= 0 ||
        w <= 0 || cout <= 0)
        return 0;
    if (x->c0 % 4 || cout % 4) return 0;
    const int64_t M = (int64_t)n * h * w;
    if (!fits_i32(M, x->c0) || !fits_i32(4 * M, cout)) return 0;
    return (int)cdiv(M, convt_bnpart_bm(M, x->c0));
}

namespace {
int convt_bwd_data_bnstats(const unet_view* x, int n, int h, int w, int cout, const float* kernel,
                           const unsigned short* kernel_x3t, const float* dout, float* dx, const float* mean,
                           const float* rstd, float* bn_partials, unet_stream_t stream) {
    if (check_view(x, "unet_conv_transpose2x2_bwd_data_bnstats")) return -1;
    const int S = unet_conv_transpose2x2_bwd_data_bnstats_slabs(x, n, h, w, cout);
    UNET_CHECK_ARG(S > 0, "unet_conv_transpose2x2_bwd_data_bnstats: needs a BNRELU view (dropout rate in [0, 1)) "
                          "and channel counts divisible by 4");
    UNET_CHECK_ARG(kernel && dout && dx && bn_partials && x->scale0 && x->shift0,
                   "unet_conv_transpose2x2_bwd_data_bnstats: bad args");
    UNET_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "unet_conv_transpose2x2_bwd_data_bnstats: mean/rstd go together");
    const int cin = x->c0;
    RowsArgs a{};
    a.a = plain_view(dout, cout);
    a.M = (int64_t)n * h * w;
    a.K = 4 * cout;
    a.uH = h;
    a.uW = w;
    a.uf = cout;
    a.B = kernel;
    // (split-precision route only where the partials are per 128-row tile, as the _slabs query said)
    a.Bx = convt_bnpart_bm(a.M, cin) == 128 ? kernel_x3t : nullptr;
    a.sbk = cin;
    a.sbn = 1;
    a.N = cin;
    a.C = dx;
    a.ldc = cin;
    a.z = x->src0;
    a.bsc = x->scale0;
    a.bsh = x->shift0;
    a.bmu = mean;
    a.brs = rstd;
    a.bnpart = bn_partials;
    // a dropout view (the bottleneck output, u_net.py:77-78): the partials are those of the
    // BN + ReLU backward of g = da * mask, as unet_bn_relu_bwd_stats forms them
    a.ep_rate = x->drop_rate;
    a.ep_inv_keep = x->drop_rate > 0.f ? 1.0f / (1.0f - x->drop_rate) : 1.0f;
    a.ep_seed = x->drop_seed;
    UNET_CHECK_ARG(rows_vec_ok(a, A_UNSHUFFLE) && ((uintptr_t)dx | (uintptr_t)x->src0) % 16 == 0,
                   "unet_conv_transpose2x2_bwd_data_bnstats: operands must be 16-B aligned");
    return launch_rows<A_UNSHUFFLE, false, E_BNPART>(a, as_stream(stream), "unet_conv_transpose2x2_bwd_data_bnstats");
}
}  // namespace

extern "C" int unet_conv_transpose2x2_bwd_data_bnstats(const unet_view* x, int n, int h, int w, int cout,
                                                       const float* kernel, const float* dout, float* dx,
                                                       const float* mean, const float* rstd, float* bn_partials,
                                                       unet_stream_t stream) {
    return convt_bwd_data_bnstats(x, n, h, w, cout, kernel, nullptr, dout, dx, mean, rstd, bn_partials, stream);
}
extern "C" int unet_conv_transpose2x2_bwd_data_bnstats_x3(const unet_view* x, int n, int h, int w, int cout,
                                                          const float* kernel, const unsigned short* kernel_x3t,
                                                          const float* dout, float* dx, const float* mean,
                                                          const float* rstd, float* bn_partials, unet_stream_t stream) {
    UNET_CHECK_ARG(kernel_x3t && (uintptr_t)kernel_x3t % 16 == 0,
                   "unet_conv_transpose2x2_bwd_data_bnstats_x3: kernel_x3t must be a 16-B aligned plane set");
    return convt_bwd_data_bnstats(x, n, h, w, cout, kernel, kernel_x3t, dout, dx, mean, rstd, bn_partials, stream);
}

namespace unet {
// head dW = sum_m x(m, k) dlogit(m, c): used by head.hip
int head_wgrad(const unet_view* x, int64_t M, const float* dlogit, int ncls, float* dkernel, void* ws, size_t ws_bytes,
               hipStream_t st) {
    WgradArgs a{};
    a.a = make_dview(*x);
    a.P = x->c0;
    a.b = plain_view(dlogit, ncls);
    a.Q = ncls;
    a.M = M;
    return run_wgrad(a, x->mode == UNET_VIEW_BNRELU ? W_BNRELU : W_PLAIN, W_PLAIN, dkernel, ws, ws_bytes, st,
                     "unet_head_bwd(filter)");
}
size_t head_wgrad_workspace(int64_t M, int cin, int ncls) { return wgrad_workspace(M, cin, ncls); }
}  // namespace unet
