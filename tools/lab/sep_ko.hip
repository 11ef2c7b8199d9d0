#include "sepconv.hip"
namespace unet {
namespace {
// ------------------------------------------------------------------------------------------
// Register-A schedule.  The MFMA A operand (the depthwise output) is computed by each lane in
// registers, straight in v_mfma_f32_32x32x2_f32's operand layout, from the staged halo: lane l of
// wave w owns GEMM row w*32 + (l & 31), i.e. pixel (2w + ((l & 31) >> 4), l & 15) of the 8 x 16
// tile, and for k-group g of a stage (8 channels) the 4 channels 8g + 4(l >> 5) + s, s = 0..3, so
// one ds_read_b128 of the halo per tap gives the 4 k-slots of 4 consecutive MFMA steps (the
// k-slot permutation of gemm_rows_vec: MFMA step s takes channels 8g + s and 8g + 4 + s).
// Each wave owns 32 rows x all BN columns, so every depthwise value is computed once per block
// and no A tile goes through LDS: there is no depthwise -> MFMA hand-off inside a stage, only the
// halo / B staging ring (double buffered, ONE barrier per 16-channel stage).  The 36 depthwise
// FMAs and 18 + BN/32 LDS reads of a k-group issue in the gaps of its 4 * BN/32 MFMAs.
//   LDS: halo [2][10*18 px][20] (16 channels + 4 pad: conflict-free b128 taps), taps [2][9][16],
//        B k-major [2][16][BN+4] (n contiguous: the staging stores are conflict-free float4s; the
//        fragment of a tile and k-group is 4 conflict-free ds_read_b32 down a column).  An n-major
//        image would give one b128 per fragment but its transposed staging stores are 16-way bank
//        conflicted (measured: that alone cost more than the whole MFMA work of the kernel).
                 // halo pixel stride (floats)


template <int MODE, bool DROP, int EPI, int BN, bool WRITE_Y, int KO>
__global__ __launch_bounds__(256, 2) void sepconv_ko_kernel(SepArgs g) {
    constexpr int TN = BN / 32;                 // MFMA tiles per wave (all BN columns)
    constexpr int NH = HPIX * (BK / 4);         // halo float4 per stage (720)
    constexpr int HR = (NH + 255) / 256;        // per thread (3)
    constexpr int NP = MODE == UNET_VIEW_POOL_BNRELU ? 4 : 1;
    constexpr int BQ = BN * (BK / 4) / 256;     // B float4 per thread per stage
    constexpr int LB = BN + 4;                  // k-major B row stride
    __shared__ __attribute__((aligned(16))) float Xs[2][HPIX * RX];
    __shared__ __attribute__((aligned(16))) float Ks[2][9 * BK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * LB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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

    // ---- halo staging geometry (fixed per thread): element e = tid + 256 j is halo pixel e >> 2,
    // channel quad e & 3 of the stage
    const int hq = tid & 3;
    int lp[HR], sp[HR];
#pragma unroll
    for (int j = 0; j < HR; ++j) {
        const int e = tid + 256 * j;
        const int pix = e >> 2, r = pix / HWp, cc = pix - r * HWp;
        const int hh = h0 - 1 + r, ww = w0 - 1 + cc;
        const bool ok = e < NH && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
        lp[j] = ok ? (n * g.H + hh) * g.W + ww : -1;
        if constexpr (MODE == UNET_VIEW_POOL_BNRELU)
            sp[j] = ok ? (n * 2 * g.H + 2 * hh) * (2 * g.W) + 2 * ww : 0;
        else
            sp[j] = ok ? lp[j] : 0;
    }
    float4 hx[HR][NP];
    float4 hsc, hsh, htap;
    int hc = 0;
    bool hbn = false;
    auto load_halo = [&](int k0) {
        const int c = k0 + 4 * hq;
        hc = c;
        const bool cok = c < Cin;
        const float* src = g.x.src0;
        int cs = g.x.c0, ci = cok ? c : 0;
        const float* scp = g.x.sc0;
        const float* shp = g.x.sh0;
        bool bn = MODE == UNET_VIEW_BNRELU || MODE == UNET_VIEW_POOL_BNRELU;
        if constexpr (MODE == UNET_VIEW_CONCAT) {
            if (ci >= g.x.c0) {
                src = g.x.src1;
                cs = g.x.c1;
                ci -= g.x.c0;
                scp = g.x.sc1;
                shp = g.x.sh1;
                bn = true;
            }
        }
        hbn = bn;
        if constexpr (MODE != UNET_VIEW_PLAIN) {
            hsc = bn ? ld4(scp + ci) : f4(1.f);
            hsh = bn ? ld4(shp + ci) : f4(0.f);
        }
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const float* b = src + (sp[j] * cs + ci);
            hx[j][0] = ld4(b);
            if constexpr (NP == 4) {
                const int rs = 2 * g.W * cs;
                hx[j][1] = ld4(b + cs);
                hx[j][2] = ld4(b + rs);
                hx[j][3] = ld4(b + rs + cs);
            }
        }
        const int tq = tid < 9 * (BK / 4) ? tid : 0;
        const int tp = tq / (BK / 4), c2 = k0 + 4 * (tq % (BK / 4));
        htap = ld4(g.dk + tp * Cin + (c2 < Cin ? c2 : 0));
    };
    auto store_halo = [&](int buf) {
        const bool cok = hc < Cin;
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const int e = tid + 256 * j;
            float4 v = hx[j][0];
            if constexpr (NP == 4) {
                v = fma4(v, hsc, hsh);
                v = max4(v, fma4(hx[j][1], hsc, hsh));
                v = max4(v, fma4(hx[j][2], hsc, hsh));
                v = max4(v, fma4(hx[j][3], hsc, hsh));
                v = relu4(v);
            } else if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (hbn) v = bnrelu4(v, hsc, hsh);
            }
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)(lp[j] < 0 ? 0 : lp[j]) * C + hc;
                v = mul4(v, drop_mult4(g.x.seed, i, g.x.rate, g.x.inv_keep));
            }
            if (lp[j] < 0 || !cok) v = f4(0.f);
            if (e < NH) *reinterpret_cast<float4*>(&Xs[buf][(e >> 2) * RX + 4 * (e & 3)]) = v;
        }
        if (tid < 9 * (BK / 4)) {
            const int c2 = hc - 4 * hq + 4 * (tid % (BK / 4));
            *reinterpret_cast<float4*>(&Ks[buf][4 * tid]) = c2 < Cin ? htap : f4(0.f);
        }
    };
    // ---- B staging: thread loads float4 (k-row, n-quad) of the n-contiguous weights
    float4 rb[BQ];
    bool bok[BQ];
    constexpr int NQ = BN / 4;
    const int bq_k = tid / NQ, bq_n = tid % NQ;
    auto load_b = [&](int k0) {
#pragma unroll
        for (int r = 0; r < BQ; ++r) {
            const int kk = k0 + bq_k + (256 / NQ) * r, nn = n0 + 4 * bq_n;
            bok[r] = kk < Cin && nn < g.Cout;
            rb[r] = ld4(g.pk + (bok[r] ? (int64_t)kk * g.Cout + nn : 0));
        }
    };
    auto store_b = [&](int buf) {
#pragma unroll
        for (int r = 0; r < BQ; ++r)
            *reinterpret_cast<float4*>(&Bs[buf][(bq_k + (256 / NQ) * r) * LB + 4 * bq_n]) = bok[r] ? rb[r] : f4(0.f);
    };

    // ---- this lane's pixel: tile row 2 wave + (lo >> 4), column lo & 15
    const int pr = 2 * wave + (lo >> 4), pc = lo & 15;
    const int xoff = (pr * HWp + pc) * RX + 4 * hi;  // halo tap (0, 0) of k-group 0
    float* yrow = nullptr;
    if constexpr (WRITE_Y) yrow = g.y + ((int64_t)(n * g.H + h0 + pr) * g.W + w0 + pc) * Cin + 4 * hi;

    floatx16 acc[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tn][r] = 0.f;

    auto compute_stage = [&](int buf, int k0) {
        const float* X = Xs[buf];
        const float* Kt = Ks[buf];
        const float* Bb = Bs[buf];
        float4 ys[BK / 8];
#pragma unroll
        for (int kg = 0; kg < BK / 8; ++kg) {
            float4 a = f4(0.f);
#pragma unroll
            for (int dy = (KO & 2) ? 1 : 0; dy < ((KO & 2) ? 2 : 3); ++dy)
#pragma unroll
                for (int dx = (KO & 2) ? 1 : 0; dx < ((KO & 2) ? 2 : 3); ++dx) {
                    const float4 xv = *reinterpret_cast<const float4*>(&X[xoff + (dy * HWp + dx) * RX + 8 * kg]);
                    const float4 kv = *reinterpret_cast<const float4*>(&Kt[(dy * 3 + dx) * BK + 8 * kg + 4 * hi]);
                    a = fma4(xv, kv, a);
                }
            ys[kg] = a;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const float* bp = &Bb[(8 * kg + 4 * hi) * LB + tn * 32 + lo];
                const float4 bf = make_float4(bp[0], bp[LB], bp[2 * LB], bp[3 * LB]);
                if constexpr (!(KO & 1)) {
                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bf.x, acc[tn], 0, 0, 0);
                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bf.y, acc[tn], 0, 0, 0);
                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bf.z, acc[tn], 0, 0, 0);
                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bf.w, acc[tn], 0, 0, 0);
                } else { acc[tn][0] += a.x * bf.x + a.w * bf.w; }
            }
            // keep the scheduler from hoisting the next k-group's 18 + TN LDS reads above these
            // MFMAs (it would hold ~90 more VGPRs and spill the 256-wide tile)
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (WRITE_Y && !(KO & 16)) {  // y for the pointwise weight gradient, after the stage's MFMAs
            if (blockIdx.y == 0) {
#pragma unroll
                for (int kg = 0; kg < BK / 8; ++kg)
                    if (k0 + 8 * kg + 4 * hi < Cin) st4(yrow + k0 + 8 * kg, ys[kg]);
            }
        }
    };

    const int nk = (KO & 64) ? 1 : (Cin + BK - 1) / BK;
    load_halo(0);
    load_b(0);
    store_halo(0);
    store_b(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        // loads past the last stage come from clamped addresses and are never stored: the loop
        // body stays branch-free around the loads
        if constexpr (!(KO & 4)) {
        load_halo((kt + 1) * BK);
        load_b((kt + 1) * BK);
        }
        compute_stage(buf, kt * BK);
        if (kt + 1 < nk) {
            store_halo(buf ^ 1);
            store_b(buf ^ 1);
        }
        if constexpr (!(KO & 8)) __syncthreads();
    }

    // ---- epilogue: row p of the tile = pixel (h0 + p / 16, w0 + p % 16); this wave's rows are
    // wave * 32 + acc_row(r, hi)
    const int64_t mbase = (int64_t)(n * g.H + h0) * g.W + w0;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
        const int col = n0 + tn * 32 + lo;
        if (col >= g.Cout || (KO & 32)) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int p = wave * 32 + acc_row(r, hi);
            g.z[(mbase + (int64_t)(p >> 4) * g.W + (p & 15)) * g.Cout + col] = acc[tn][r];
        }
    }
    if constexpr (EPI == E_STATS) {
        // per column (mean, M2) of the tile's 128 rows: per-wave sums, a fixed-order combine of
        // the 4 waves through LDS (the loop ended on a barrier, so Bs is free)
        float* red = &Bs[0][0];
        float mean[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) s += acc[tn][r];
            s += __shfl_xor(s, 32, 64);
            if (hi == 0) red[wave * BN + tn * 32 + lo] = s;
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int cl = tn * 32 + lo;
            mean[tn] = ((red[cl] + red[BN + cl]) + (red[2 * BN + cl] + red[3 * BN + cl])) * (1.0f / 128.0f);
        }
        __syncthreads();
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            float q = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float d = acc[tn][r] - mean[tn];
                q = fmaf(d, d, q);
            }
            q += __shfl_xor(q, 32, 64);
            if (hi == 0) red[wave * BN + tn * 32 + lo] = q;
        }
        __syncthreads();
        if (wave == 0 && hi == 0) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int cl = tn * 32 + lo;
                const int col = n0 + cl;
                if (col < g.Cout)
                    g.stats[(int64_t)blockIdx.x * g.Cout + col] =
                        make_float2(mean[tn], (red[cl] + red[BN + cl]) + (red[2 * BN + cl] + red[3 * BN + cl]));
            }
        }
    }
}

}
}
