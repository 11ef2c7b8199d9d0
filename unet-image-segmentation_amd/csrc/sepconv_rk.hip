// Fused SeparableConv2D forward, register-A schedule (reference model/u_net.py:14-23).
// Built without SLP vectorisation (Makefile): packed f32 VALU beside MFMAs stalls the matrix
// pipe (MI355X_MICROARCH.md, "price of one filler beside MFMAs"), so the depthwise FMAs stay scalar.
#include "sepconv.h"

namespace unet {
namespace sep {
namespace {

// ------------------------------------------------------------------------------------------
// Register-A schedule.  The MFMA A operand (the depthwise output) is computed by each lane in
// registers, straight in v_mfma_f32_32x32x2_f32's operand layout, from the staged halo: lane l of
// wave w owns GEMM row w*32 + (l & 31), i.e. pixel (2w + (lo >> 4), rk_col(lo)) of the 8 x 16
// tile (lo = l & 31; the second pixel row is rotated by two columns so that every 16-lane group of
// a ds_read_b128 halo tap covers the 64 banks once: rows are 18 halo pixels apart, and without the
// rotation two lanes of each group share a bank), and for k-group g of a stage (8 channels) the 4
// channels 8g + 4(l >> 5) + s, s = 0..3, so
// one ds_read_b128 of the halo per tap gives the 4 k-slots of 4 consecutive MFMA steps (the
// k-slot permutation of gemm_rows_vec: MFMA step s takes channels 8g + s and 8g + 4 + s).
// Each wave owns 32 rows x all BN columns, so every depthwise value is computed once per block
// and no A tile goes through LDS: there is no depthwise -> MFMA hand-off inside a stage, only the
// halo / B staging ring (three slots, ONE barrier per 16-channel stage).  The depthwise of the
// next k-group (36 FMAs, 18 LDS reads) is interleaved with the MFMAs of the current one.
//   LDS (one buffer; the epilogue reuses it): halo [3][10*18 px][20] (16 channels + 4 pad), taps [3][9][16],
//        B k-major [3][16][BN+4] (n contiguous: the staging stores are conflict-free float4s; the
//        fragment of a tile and k-group is 4 conflict-free ds_read_b32 down a column).  An n-major
//        image would give one b128 per fragment but its transposed staging stores are 16-way bank
//        conflicted (measured: that alone cost more than the whole MFMA work of the kernel).
//   Epilogue: each wave writes its 32 x BN accumulator tile into LDS and reads it back as row
//   float4s, so z leaves as 16-byte stores of BN contiguous channels per pixel (the accumulator
//   layout holds one column per lane: 4-byte stores, 2 rows x 128 B per instruction).
constexpr int RX = BK + 4;                 // halo pixel stride (floats)
constexpr int HPIX = HHp * HWp;            // 180 halo pixels

// tile column of the pixel that lane lo (0..31) of a wave owns (row 2w + (lo >> 4))
__device__ __forceinline__ int rk_col(int lo) { return lo < 16 ? lo : ((lo + 14) & 15); }
template <int BN, bool X6 = false>
struct RkLds {
    // X6: B as three bf16 planes [BN][16 k] (32-byte rows; the two 16-byte k chunks of row n are
    // swapped when bit 3 of n is set, so the fragment reads of 16-lane groups are conflict-free)
    // X6: the stage's depthwise taps live in the halo pixels' pad floats (pixel i's 4 pad floats hold
    // tap float4 i, i < 36), so a slot is 576 B smaller: at BN 128 three blocks fit a CU (3 x 53.76 KB;
    // with a separate tap buffer the 54.78 KB allocation granule allowed two)
    static constexpr int XSZ = HPIX * RX, KSZ = X6 ? 0 : 9 * BK, BSZ = X6 ? 3 * BN * BK / 2 : BK * (BN + 4);
    static constexpr int SLOTS = X6 ? 2 : 3;           // X6: two slots (53 KB: 3 blocks per CU; 79 KB at BN 256: 2)
    static constexpr int RING = SLOTS * (XSZ + KSZ + BSZ);
    static constexpr int EC = X6 && BN > 64 ? 64 : BN;  // accumulator columns per epilogue pass
    static constexpr int TLD = EC + 4;                  // epilogue transpose row stride
    static constexpr int EPI = 4 * 32 * TLD + 4 * BN;   // 4 waves' tiles + the statistics combine
    static constexpr int SIZE = RING > EPI ? RING : EPI;
};

// X6 (split precision; no max-pool views, Cin % 16 == 0): per 16-channel stage each lane evaluates
// the depthwise output of its pixel for the 8 channels 8 (l >> 5) + j of v_mfma_f32_32x32x16_bf16's
// A operand (same taps, same fmaf order: y bitwise equal), splits them into three bf16 fragments
// (common.h split4) and runs mfma_x6 against the pre-split weight planes (SepArgs::pkx) per 32-column
// tile: 6 x 32 MFMA cycles per stage and tile instead of 8 x 64.
template <int MODE, bool DROP, int EPI, int BN, bool WRITE_Y, bool X6 = false>
__global__ __launch_bounds__(256, X6 && BN <= 128 ? 3 : 2) void sepconv_rk_kernel(SepArgs g) {
    static_assert(!X6 || MODE != UNET_VIEW_POOL_BNRELU, "X6: no max-pool views");
    constexpr int TN = BN / 32;                 // MFMA tiles per wave (all BN columns)
    constexpr int NH = HPIX * (BK / 4);         // halo float4 per stage (720)
    constexpr int HR = (NH + 255) / 256;        // per thread (3)
    constexpr int NP = MODE == UNET_VIEW_POOL_BNRELU ? 4 : 1;
    constexpr int BQ = X6 ? 1 : BN * (BK / 4) / 256;  // B float4 per thread per stage
    constexpr int LB = BN + 4;                  // k-major B row stride
    constexpr int BXN = 3 * BN * 2;             // X6: 16-byte B chunks per stage (a multiple of 64)
    using L = RkLds<BN, X6>;
    __shared__ __attribute__((aligned(16))) float smem[L::SIZE];
    auto Xs = [&](int b) { return smem + b * L::XSZ; };
    auto Ks = [&](int b) { return smem + L::SLOTS * L::XSZ + b * L::KSZ; };
    auto Bs = [&](int b) { return smem + L::SLOTS * (L::XSZ + L::KSZ) + b * L::BSZ; };

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    const int tiles_w = g.W / TW, tiles_h = g.H / TH;
    // pixel tile: XCD-contiguous order (neighbouring tiles re-read each other's halo through one L2;
    // the tile count is a multiple of 8 on every level the fused forward runs)
    const int tile = (gridDim.x & 7) == 0 ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    int t = tile;
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
            if (e < NH) *reinterpret_cast<float4*>(&Xs(buf)[(e >> 2) * RX + 4 * (e & 3)]) = v;
        }
        if (tid < 9 * (BK / 4)) {
            const int c2 = hc - 4 * hq + 4 * (tid % (BK / 4));
            float* td = X6 ? &Xs(buf)[tid * RX + BK] : &Ks(buf)[4 * tid];  // X6: pixel tid's pad
            *reinterpret_cast<float4*>(td) = c2 < Cin ? htap : f4(0.f);
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
            *reinterpret_cast<float4*>(&Bs(buf)[(bq_k + (256 / NQ) * r) * LB + 4 * bq_n]) = bok[r] ? rb[r] : f4(0.f);
    };
    // X6 B staging by LDS-DMA (global_load_lds_dwordx4, no VGPR destination): LDS chunk q = 64 i + lane
    // of a slot is (row q >> 1 = plane * BN + column, k half (q & 1) ^ bit 3 of the column) -- the
    // image is lane-linear, so the conflict-free swizzle goes on the source address.  Wave w issues
    // wave-instructions i = w, w + 4, ... of the stage's BXN / 64.  Columns past Cout load column 0
    // (finite data; their accumulators are never stored); k always lies inside Cin (Cin % 16 == 0).
    // Issued from inline asm: hipcc's wait bookkeeping would put vmcnt(0) before every ds_read while
    // a DMA it knows of is in flight; the kernel waits for it itself (dma_wait).
    constexpr int NIW = (BXN / 64 + 3) / 4;     // DMA wave-instructions per wave and stage
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    int bxo[X6 ? NIW : 1];
#pragma unroll
    for (int j = 0; j < (X6 ? NIW : 1); ++j) {
        const int q = (wv + 4 * j) * 64 + lane, row = q >> 1, pl = row / BN, nn = row - pl * BN;
        const int c = (q & 1) ^ ((nn >> 3) & 1), col = n0 + nn < g.Cout ? n0 + nn : 0;
        bxo[j] = (pl * g.Cout + col) * Cin + 8 * c;
    }
    auto dma_bx = [&](int k0, int buf) {
        const unsigned base = (unsigned)(uintptr_t)(lds_void*)Bs(buf);
#pragma unroll
        for (int j = 0; j < NIW; ++j) {
            const int i = wv + 4 * j;
            if ((BXN / 64) % 4 == 0 || i < BXN / 64) {
                const unsigned short* src = g.pkx + bxo[j] + k0;
                const unsigned dst = base + i * 1024;
                unsigned keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
            }
        }
    };
    // every vector-memory operation of this wave retired (the DMA, and the stage's y stores)
    auto dma_wait = [] { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

    // ---- this lane's pixel: tile row 2 wave + (lo >> 4), column rk_col(lo)
    const int pr = 2 * wave + (lo >> 4), pc = rk_col(lo);
    const int xoff = (pr * HWp + pc) * RX + 4 * hi;  // halo tap (0, 0) of k-group 0
    float* yrow = nullptr;
    if constexpr (WRITE_Y) yrow = g.y + ((int64_t)(n * g.H + h0 + pr) * g.W + w0 + pc) * Cin + 4 * hi;

    floatx16 acc[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tn][r] = 0.f;

    // depthwise output of k-group kg (this lane's pixel, 4 channels) from halo / tap buffer b
    auto dw = [&](int b, int kg) {
        const float* X = Xs(b);
        const float* Kt = Ks(b);
        float4 a = f4(0.f);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const float4 xv = *reinterpret_cast<const float4*>(&X[xoff + (dy * HWp + dx) * RX + 8 * kg]);
                const float4 kv = *reinterpret_cast<const float4*>(&Kt[(dy * 3 + dx) * BK + 8 * kg + 4 * hi]);
                a = fma4(xv, kv, a);
            }
        return a;
    };
    // the 4 * TN MFMAs of k-group kg with A = a, and (independent of them) the depthwise of the
    // NEXT k-group (buffer nb, group nkg): interleaved one MFMA : two LDS reads : two VALU ops, so
    // the depthwise runs in the MFMA pipe's shadow instead of between MFMA bursts
    auto mfma_dw = [&](const float4 a, int b, int kg, int nb, int nkg) {
        const float* Bb = Bs(b);
        float4 bf[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const float* bp = &Bb[(8 * kg + 4 * hi) * LB + tn * 32 + lo];
            bf[tn] = make_float4(bp[0], bp[LB], bp[2 * LB], bp[3 * LB]);
        }
        const float4 an = dw(nb, nkg);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bf[tn].x, acc[tn], 0, 0, 0);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bf[tn].y, acc[tn], 0, 0, 0);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bf[tn].z, acc[tn], 0, 0, 0);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bf[tn].w, acc[tn], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4 * TN; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 LDS reads
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // 2 VALU
        }
        __builtin_amdgcn_sched_barrier(0);
        return an;
    };

    // Three-slot ring (halo, taps, B): stage kt computes from slot kt % 3 and already evaluates
    // the depthwise of stage kt+1's first k-group from slot (kt+1) % 3 (staged one stage ahead),
    // while the global loads of stage kt+2 are in flight; they are written into slot (kt+2) % 3,
    // last read during stage kt-1.  One barrier per stage.
    const int nk = (Cin + BK - 1) / BK;
    if constexpr (X6) {
        // depthwise of this lane's pixel, channels 8 hi + 0..7 of the stage, from halo / taps b
        const int xoff8 = (pr * HWp + pc) * RX + 8 * hi;
        auto dw8 = [&](int b, float4& o0, float4& o1) {
            const float* X = Xs(b);
            o0 = f4(0.f);
            o1 = f4(0.f);
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const float* xp = &X[xoff8 + (dy * HWp + dx) * RX];
                    // tap float4 (dy * 3 + dx) * 4 + 2 hi (+ 1): the pads of those halo pixels
                    const float* kp = &X[((dy * 3 + dx) * 4 + 2 * hi) * RX + BK];
                    o0 = fma4(*reinterpret_cast<const float4*>(xp), *reinterpret_cast<const float4*>(kp), o0);
                    o1 = fma4(*reinterpret_cast<const float4*>(xp + 4), *reinterpret_cast<const float4*>(kp + RX), o1);
                }
        };
        float* yrow8 = nullptr;
        if constexpr (WRITE_Y) yrow8 = g.y + ((int64_t)(n * g.H + h0 + pr) * g.W + w0 + pc) * Cin + 8 * hi;
        // stage kt computes from slot kt % 2 while stage kt + 1's loads (issued before it) land;
        // they are written to the other slot after the compute, then stage kt + 2's are issued.
        // Only stage 0's loads are exposed (one latency per block, not two: at 4-8 stages per
        // block that is most of the prologue)
        // B: stage kt + 1's planes are DMA'd into the other slot at the top of stage kt (free since
        // the barrier that ended stage kt - 1: its lgkmcnt(0) retired the slot's fragment reads);
        // dma_wait after store_halo -- before stage kt + 2's halo loads are issued -- retires them
        // ahead of the stage's barrier, the only thing that orders them for the next stage's reads
        load_halo(0);
        dma_bx(0, 0);
        store_halo(0);
        dma_wait();
        if (nk > 1) load_halo(BK);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const int cb = kt & 1, wb = cb ^ 1;
            if (kt + 1 < nk) dma_bx((kt + 1) * BK, wb);
            // this stage's depthwise (VALU), then its MFMAs: with two waves per SIMD one wave's
            // depthwise runs beside the other's MFMAs (a look-ahead inside the wave needed ~60 more
            // registers and spilled)
            float4 a0, a1;
            dw8(cb, a0, a1);
            if constexpr (WRITE_Y) {
                const int k0 = kt * BK;
                if (blockIdx.y == 0 && k0 < Cin) {
                    st4(yrow8 + k0, a0);
                    st4(yrow8 + k0 + 4, a1);
                }
            }
            bf16x8 af[3];
            {
                const Split4 s0 = split4(a0), s1 = split4(a1);
                af[0] = __builtin_bit_cast(bf16x8, make_uint4(s0.h.x, s0.h.y, s1.h.x, s1.h.y));
                af[1] = __builtin_bit_cast(bf16x8, make_uint4(s0.m.x, s0.m.y, s1.m.x, s1.m.y));
                af[2] = __builtin_bit_cast(bf16x8, make_uint4(s0.l.x, s0.l.y, s1.l.x, s1.l.y));
            }
            const unsigned short* Bb = reinterpret_cast<const unsigned short*>(Bs(cb));
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int nn = tn * 32 + lo;
                const int cs = hi ^ ((nn >> 3) & 1);
                bf16x8 bfr[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    bfr[pl] = *reinterpret_cast<const bf16x8*>(Bb + (pl * BN + nn) * BK + 8 * cs);
                acc[tn] = mfma_x6(af, bfr, acc[tn]);
            }
            if (kt + 1 < nk) {
                store_halo(wb);
                dma_wait();
                if (kt + 2 < nk) load_halo((kt + 2) * BK);
            }
            __syncthreads();
        }
    } else {
    load_halo(0);
    load_b(0);
    store_halo(0);
    store_b(0);
    load_halo(BK);
    load_b(BK);
    store_halo(1);
    store_b(1);
    __syncthreads();
    float4 a = dw(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int cb = kt % 3, nb = (kt + 1) % 3, wb = (kt + 2) % 3;
        // loads past the last stage come from clamped addresses and are never stored: the loop
        // body stays branch-free around the loads; the last stage's look-ahead depthwise reads a
        // stale (valid) slot and is discarded
        load_halo((kt + 2) * BK);
        load_b((kt + 2) * BK);
        const float4 a1 = mfma_dw(a, cb, 0, cb, 1);
        const float4 a0 = mfma_dw(a1, cb, 1, nb, 0);
        if constexpr (WRITE_Y) {  // y (depthwise output) for the pointwise weight gradient
            const int k0 = kt * BK;
            if (blockIdx.y == 0) {
                if (k0 + 4 * hi < Cin) st4(yrow + k0, a);
                if (k0 + 8 + 4 * hi < Cin) st4(yrow + k0 + 8, a1);
            }
        }
        a = a0;
        if (kt + 2 < nk) {
            store_halo(wb);
            store_b(wb);
        }
        __syncthreads();
    }
    }

    // ---- epilogue (the loop ended on a barrier: the ring is free).  Accumulator row
    // acc_row(r, hi) of wave w is tile pixel (2w + (row >> 4), rk_col(row)).  The accumulator
    // tile leaves through LDS in EC-column passes (X6: 64, so the epilogue fits the two-slot ring)
    constexpr int EC = L::EC, TLD = L::TLD;
    float* T = smem + wave * 32 * TLD;
    float* red = smem + 4 * 32 * TLD;
    if constexpr (EPI == E_STATS) {
        // per column (mean, M2) of the tile's 128 rows: per-wave sums, a fixed-order combine of
        // the 4 waves through LDS
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
                    g.stats[(int64_t)tile * g.Cout + col] =
                        make_float2(mean[tn], (red[cl] + red[BN + cl]) + (red[2 * BN + cl] + red[3 * BN + cl]));
            }
        }
    }
    constexpr int Q4 = EC / 4, NS = 32 * Q4 / 64;
#pragma unroll
    for (int hp = 0; hp < BN / EC; ++hp) {
        const int cbase = n0 + hp * EC;  // first output channel of this pass
        __syncthreads();                 // (the statistics' / previous pass's LDS reads are done)
#pragma unroll
        for (int tn = 0; tn < EC / 32; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r) T[acc_row(r, hi) * TLD + tn * 32 + lo] = acc[hp * (EC / 32) + tn][r];
        __syncthreads();
        if (g.zsel) {
            // the wave's two pixel rows hold 8 whole 2x2 windows: their pooling selection (zsel) for
            // the next stage's max-pool view.  T row of pixel (sub, col): col, or 16 + ((col + 2) & 15)
            // on the second row (rk_col's rotation inverted)
            constexpr int NP4 = 8 * Q4 / 64;
#pragma unroll
            for (int i = 0; i < NP4; ++i) {
                const int idx = i * 64 + lane, j = idx / Q4, q = idx - j * Q4;
                const int c0 = 2 * j, c1 = 2 * j + 1;
                const float4 a = *reinterpret_cast<const float4*>(&T[c0 * TLD + 4 * q]);
                const float4 b = *reinterpret_cast<const float4*>(&T[c1 * TLD + 4 * q]);
                const float4 c = *reinterpret_cast<const float4*>(&T[(16 + ((c0 + 2) & 15)) * TLD + 4 * q]);
                const float4 d = *reinterpret_cast<const float4*>(&T[(16 + ((c1 + 2) & 15)) * TLD + 4 * q]);
                const int col = cbase + 4 * q;
                if (col < g.Cout) {
                    const float4 gm = g.gamma ? ld4(g.gamma + col) : f4(0.f);
                    float4 o;
                    o.x = pool_sel(a.x, b.x, c.x, d.x, signbit(gm.x));
                    o.y = pool_sel(a.y, b.y, c.y, d.y, signbit(gm.y));
                    o.z = pool_sel(a.z, b.z, c.z, d.z, signbit(gm.z));
                    o.w = pool_sel(a.w, b.w, c.w, d.w, signbit(gm.w));
                    const int H2 = g.H >> 1, W2 = g.W >> 1;
                    st4(g.zsel + ((int64_t)(n * H2 + (h0 >> 1) + wave) * W2 + (w0 >> 1) + j) * g.Cout + col, o);
                }
            }
        }
        // z: the wave's 32 pixels x EC channels as float4s (EC / 4 per pixel, 64 per instruction)
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int idx = i * 64 + lane, row = idx / Q4, q = idx - row * Q4;
            const float4 v = *reinterpret_cast<const float4*>(&T[row * TLD + 4 * q]);
            const int ph = h0 + 2 * wave + (row >> 4), pw = w0 + rk_col(row);
            if (cbase + 4 * q < g.Cout) st4(g.z + ((int64_t)(n * g.H + ph) * g.W + pw) * g.Cout + cbase + 4 * q, v);
        }
    }
}

template <int MODE, bool DROP, int BN, bool X6>
void launch_rk_x(const SepArgs& a, bool stats, bool write_y, hipStream_t st) {
    const dim3 grid((unsigned)(a.N * (a.H / TH) * (a.W / TW)), (unsigned)cdiv(a.Cout, BN));
    if (stats) {
        if (write_y) sepconv_rk_kernel<MODE, DROP, E_STATS, BN, true, X6><<<grid, 256, 0, st>>>(a);
        else sepconv_rk_kernel<MODE, DROP, E_STATS, BN, false, X6><<<grid, 256, 0, st>>>(a);
    } else {
        if (write_y) sepconv_rk_kernel<MODE, DROP, E_STORE, BN, true, X6><<<grid, 256, 0, st>>>(a);
        else sepconv_rk_kernel<MODE, DROP, E_STORE, BN, false, X6><<<grid, 256, 0, st>>>(a);
    }
}

template <int MODE, bool DROP, int BN>
void launch_rk_x6(const SepArgs& a, bool stats, bool write_y, hipStream_t st) {
    if constexpr (MODE != UNET_VIEW_POOL_BNRELU) launch_rk_x<MODE, DROP, BN, true>(a, stats, write_y, st);
}

template <int MODE, bool DROP, int BN>
void launch_rk_t(const SepArgs& a, bool stats, bool write_y, hipStream_t st) {
    if constexpr (MODE != UNET_VIEW_POOL_BNRELU) {
        if (a.pkx && rk_x6_supported(MODE, a.Cin)) {
            launch_rk_x<MODE, DROP, BN, true>(a, stats, write_y, st);
            return;
        }
    }
    launch_rk_x<MODE, DROP, BN, false>(a, stats, write_y, st);
}

}  // namespace

bool rk_x6_supported(int mode, int cin) { return mode != UNET_VIEW_POOL_BNRELU && cin % 16 == 0 && cin >= 64; }

bool rk_supported(int mode, int cin, int cout) {
    // max-pool views only up to 128 output channels: wider layers keep the LDS-A-tile kernel's
    // 256-wide 8-wave tile, which pools each halo element once for all columns (measured:
    // tools/lab/sep_rk_lab.hip, enc3_block1 / enc4_block1)
    return mode >= UNET_VIEW_PLAIN && mode <= UNET_VIEW_CONCAT && cin >= 64 && cout >= 64 &&
           (mode != UNET_VIEW_POOL_BNRELU || cout <= 128);
}

int launch_rk(const SepArgs& a, int mode, bool drop, bool stats, bool write_y, hipStream_t st) {
    if (!rk_supported(mode, a.Cin, a.Cout)) return -1;
    // split precision with >= 256 outputs: one 256-column tile (two blocks per CU), so the
    // depthwise and its halo are evaluated once per pixel tile instead of once per 128 columns,
    // and the 64 x 64 level's 512 pixel tiles fill the 512 block slots in one round
    const bool x6 = a.pkx && rk_x6_supported(mode, a.Cin);
    const int bn = a.Cout <= 64 ? 64 : (x6 && a.Cout >= 256 ? 256 : 128);
#define UNET_RK(M, D)                                                          \
    do {                                                                       \
        if (bn == 64) launch_rk_t<M, D, 64>(a, stats, write_y, st);            \
        else if (bn == 128) launch_rk_t<M, D, 128>(a, stats, write_y, st);     \
        else launch_rk_x6<M, D, 256>(a, stats, write_y, st);                   \
    } while (0)
    switch (mode) {
        case UNET_VIEW_PLAIN: if (drop) UNET_RK(UNET_VIEW_PLAIN, true); else UNET_RK(UNET_VIEW_PLAIN, false); break;
        case UNET_VIEW_BNRELU: if (drop) UNET_RK(UNET_VIEW_BNRELU, true); else UNET_RK(UNET_VIEW_BNRELU, false); break;
        case UNET_VIEW_POOL_BNRELU:
            if (drop) UNET_RK(UNET_VIEW_POOL_BNRELU, true); else UNET_RK(UNET_VIEW_POOL_BNRELU, false);
            break;
        default: if (drop) UNET_RK(UNET_VIEW_CONCAT, true); else UNET_RK(UNET_VIEW_CONCAT, false); break;
    }
#undef UNET_RK
    return 0;
}

}  // namespace sep
}  // namespace unet
