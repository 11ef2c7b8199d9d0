// Fused SeparableConv2D forward (reference model/u_net.py:14-23), split-precision register-A
// schedule, PERSISTENT over pixel tiles: the short-K blocks (64 / 128 input channels, 64 / 128
// outputs: enc1_block2, enc2_block1, enc2_block2, dec1_*, dec2_block2).
//
// Why a second kernel beside sepconv_rk.hip's: with 4 or 8 k-stages per 8 x 16-pixel tile the
// one-tile-per-block kernel spends much of every block in its prologue (the first stage's halo /
// weight loads, exposed) and its epilogue (z through LDS, stores), and a stage's loads are only one
// stage ahead.  Knock-outs (tools/lab/x6_ko_lab, profiles/r4a_x6_ko.log): at batch 32 enc2_block2
// takes 292 us, 182 without the k-loop loads, 174 without the stores, 136 without both, and the
// MFMAs are completely hidden.  Here a block walks a strided sequence of tiles (the blocks of
// one XCD on a contiguous range at any time: neighbouring halos through one L2) as ONE stage stream: stage
// s + PD's global loads are issued while stage s computes, across tile boundaries, so a tile's
// first loads are in flight during the previous tile's last stages and its epilogue, and the
// z / y stores overlap the next tile's loads and MFMAs.  What is loaded once per block instead of
// once per tile: the depthwise taps (9 x Cin) and the view's BatchNorm scale / shift.
// The statistics epilogue writes per-wave (mean, M2) of 32 rows to LDS and one wave combines the
// four (Chan, fixed order) after the NEXT stage's barrier: no extra barrier per tile.  The z tile
// leaves through a per-wave LDS transpose (no block barrier).
//
// LDS (floats): halo ring 2 x [180 px][16 ch] with the channel quads of pixel P XOR-swizzled by
// (P >> 2) & 3 (rk_col's lane -> pixel map then reads conflict-free with no pad: the 16 lanes of a
// ds_read_b128 group cover 16 consecutive residues of P mod 16), B ring 2 x [3][BN][16] bf16,
// taps [9][CIN], scale / shift [2][CIN], per-wave transpose 4 x [32][36], statistics [4][BN][2].
// 58-76 KB: two blocks per CU, <= 256 VGPRs.
#include <type_traits>

#include "sepconv.h"

namespace unet {
namespace sep {
namespace {

constexpr int PX = 16;               // halo pixel stride (floats): 16 channels, swizzled quads
constexpr int PHPIX = HHp * HWp;     // 180 halo pixels
constexpr int PTLD = 36;             // epilogue transpose row stride (32 columns + 4)

__device__ __forceinline__ int px_col(int lo) { return lo < 16 ? lo : ((lo + 14) & 15); }
// float offset of channel quad q of halo pixel p
__device__ __forceinline__ int px_off(int p, int q) { return p * PX + 4 * (q ^ ((p >> 2) & 3)); }

template <int BN, int CIN>
struct PxLds {
    static constexpr int XSZ = PHPIX * PX;          // 2880
    static constexpr int BSZ = 3 * BN * BK / 2;     // bf16 planes as floats
    static constexpr int X0 = 0;
    static constexpr int B0 = X0 + 2 * XSZ;
    static constexpr int TAP0 = B0 + 2 * BSZ;
    static constexpr int AFF0 = TAP0 + 9 * CIN;
    static constexpr int T0 = AFF0 + 2 * CIN;
    static constexpr int RED0 = T0 + 4 * 32 * PTLD;
    static constexpr int SIZE = RED0 + 4 * BN * 2;
};

template <int MODE, bool DROP, bool STATS, int BN, int CIN, bool WRITE_Y, int PD>
__global__ __launch_bounds__(256, 2) void sepconv_px_kernel(SepArgs g, int ntiles) {
    static_assert(MODE == UNET_VIEW_PLAIN || MODE == UNET_VIEW_BNRELU || MODE == UNET_VIEW_CONCAT, "view");
    static_assert(PD >= 1 && PD <= 4, "prefetch depth");
    constexpr int TN = BN / 32;
    constexpr int NK = CIN / BK;
    constexpr int NH = PHPIX * (BK / 4);   // halo float4 per stage (720)
    constexpr int HR = (NH + 255) / 256;   // per thread (3)
    constexpr int BXN = 3 * BN * 2;        // 16-byte B chunks per stage
    constexpr int BXC = (BXN + 255) / 256;
    constexpr int NSET = PD;               // register staging sets (one per stage in flight)
    using L = PxLds<BN, CIN>;
    __shared__ __attribute__((aligned(16))) float smem[L::SIZE];
    float* const Xs0 = smem + L::X0;
    float* const taps = smem + L::TAP0;
    float* const aff = smem + L::AFF0;     // [0, CIN): scale, [CIN, 2 CIN): shift
    float2* const red = reinterpret_cast<float2*>(smem + L::RED0);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lo = lane & 31, hi = lane >> 5;
    const int tiles_w = g.W / TW, tiles_h = g.H / TH;
    // this block's tiles: r, r + G, r + 2 G, ... with r XCD-contiguous (blocks b, b + 8, ... share
    // an XCD), so at any time the blocks of one XCD work on a contiguous range of tiles and
    // vertically neighbouring halos meet in that XCD's L2 (a contiguous run per block instead read
    // 1.27x the algorithmic bytes: the tile above was long evicted)
    const int G = gridDim.x;
    const int r = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const int S = (r < ntiles ? (ntiles - 1 - r) / G + 1 : 0) * NK;

    // ---- once per block: depthwise taps [9][CIN] and the view's affine [2][CIN]
    for (int i = tid; i < 9 * CIN / 4; i += 256) st4(taps + 4 * i, ld4(g.dk + 4 * i));
    if constexpr (MODE != UNET_VIEW_PLAIN) {
        for (int i = tid; i < CIN / 4; i += 256) {
            const int c = 4 * i;
            float4 sc = f4(1.f), sh = f4(0.f);
            if constexpr (MODE == UNET_VIEW_BNRELU) {
                sc = ld4(g.x.sc0 + c);
                sh = ld4(g.x.sh0 + c);
            } else if (c >= g.x.c0) {
                sc = ld4(g.x.sc1 + c - g.x.c0);
                sh = ld4(g.x.sh1 + c - g.x.c0);
            }
            st4(aff + c, sc);
            st4(aff + CIN + c, sh);
        }
    }

    // zsel: the sign bits of gamma at this lane's epilogue columns (tn * 32 + 4 (lane & 7) + i ->
    // bit 4 tn + i), read once here -- a gamma load inside the tile loop's epilogue made the wave
    // wait for every load and store it had in flight (vmcnt(0)), the prefetched stages included
    unsigned gneg = 0;
    if (g.zsel && g.gamma) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const float4 gm = ld4(g.gamma + tn * 32 + 4 * (lane & 7));
            gneg |= ((signbit(gm.x) ? 1u : 0u) | (signbit(gm.y) ? 2u : 0u) | (signbit(gm.z) ? 4u : 0u) |
                     (signbit(gm.w) ? 8u : 0u)) << (4 * tn);
        }
    }
    __syncthreads();  // taps / affine visible before the first stage's staging reads them

    // ---- staging: set p holds stage s's halo (HR float4 / thread) and B chunks (BXC / thread)
    const int hq = tid & 3;
    // the weight chunks of the two sets are two NAMED arrays (as one [NSET][BXC] array hipcc left
    // them in scratch memory, whose loads' vmcnt(0) waits drained the whole prefetch)
    float4 hx[NSET][HR];
    int hl[NSET][HR];  // linear pixel index of the element, -1 outside the image
    uint4 rb0[BXC], rb1[BXC], rb2[BXC], rb3[BXC];
    auto tile_geom = [&](int tile, int& n, int& h0, int& w0) {
        const int tw = tile % tiles_w, t2 = tile / tiles_w;
        w0 = tw * TW;
        h0 = (t2 % tiles_h) * TH;
        n = t2 / tiles_h;
    };
    auto load = [&](int s, auto set) {
        constexpr int p = decltype(set)::value;
        const int i = s / NK, k0 = (s - i * NK) * BK;
        int n, h0, w0;
        tile_geom(r + i * G, n, h0, w0);
        const float* src = g.x.src0;
        int cs = g.x.c0, ci = k0 + 4 * hq;
        if constexpr (MODE == UNET_VIEW_CONCAT) {
            if (k0 >= g.x.c0) {
                src = g.x.src1;
                cs = g.x.c1;
                ci -= g.x.c0;
            }
        }
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const int e = tid + 256 * j;
            const int pix = e >> 2, rr = pix / HWp, cc = pix - rr * HWp;
            const int hh = h0 - 1 + rr, ww = w0 - 1 + cc;
            // branch-free: a clamped address, the validity kept for the LDS write
            const bool ok = ((NH % 256 == 0) | (e < NH)) & ((unsigned)hh < (unsigned)g.H) & ((unsigned)ww < (unsigned)g.W);
            const int lp = (n * g.H + hh) * g.W + ww;
            hl[p][j] = ok ? lp : -1;
            hx[p][j] = ld4(src + ((int64_t)(ok ? lp : 0) * cs + ci));
        }
#pragma unroll
        for (int j = 0; j < BXC; ++j) {
            const int e = tid + 256 * j, pl = e / (2 * BN), rm = e - pl * 2 * BN, nn = rm >> 1, c = rm & 1;
            const bool ok = (BXN % 256 == 0) | (e < BXN);
            const uint4 v = *reinterpret_cast<const uint4*>(g.pkx + (ok ? ((int64_t)pl * g.Cout + nn) * CIN + k0 + 8 * c : 0));
            if constexpr (p == 0) rb0[j] = v;
            else if constexpr (p == 1) rb1[j] = v;
            else if constexpr (p == 2) rb2[j] = v;
            else rb3[j] = v;
        }
    };
    auto store = [&](int s, int slot, auto set) {
        constexpr int p = decltype(set)::value;
        const int k0 = (s % NK) * BK;
        const int hc = k0 + 4 * hq;  // logical channel of this thread's quad
        float* X = Xs0 + slot * L::XSZ;
        bool bn = MODE == UNET_VIEW_BNRELU;
        if constexpr (MODE == UNET_VIEW_CONCAT) bn = k0 >= g.x.c0;
        float4 sc = f4(1.f), sh = f4(0.f);
        if constexpr (MODE != UNET_VIEW_PLAIN) {
            sc = *reinterpret_cast<const float4*>(aff + hc);
            sh = *reinterpret_cast<const float4*>(aff + CIN + hc);
        }
#pragma unroll
        for (int j = 0; j < HR; ++j) {
            const int e = tid + 256 * j;
            float4 v = hx[p][j];
            if constexpr (MODE != UNET_VIEW_PLAIN) {
                if (bn) v = bnrelu4(v, sc, sh);
            }
            if constexpr (DROP) {
                const uint64_t li = (uint64_t)(hl[p][j] < 0 ? 0 : hl[p][j]) * g.x.C + hc;
                v = mul4(v, drop_mult4(g.x.seed, li, g.x.rate, g.x.inv_keep));
            }
            if (hl[p][j] < 0) v = f4(0.f);
            if (NH % 256 == 0 || e < NH) st4(X + px_off(e >> 2, e & 3), v);
        }
        unsigned short* Bb = reinterpret_cast<unsigned short*>(smem + L::B0 + slot * L::BSZ);
#pragma unroll
        for (int j = 0; j < BXC; ++j) {
            const int e = tid + 256 * j, pl = e / (2 * BN), rm = e - pl * 2 * BN, nn = rm >> 1, c = rm & 1;
            uint4 v;
            if constexpr (p == 0) v = rb0[j];
            else if constexpr (p == 1) v = rb1[j];
            else if constexpr (p == 2) v = rb2[j];
            else v = rb3[j];
            if (BXN % 256 == 0 || e < BXN) *reinterpret_cast<uint4*>(Bb + (pl * BN + nn) * BK + 8 * (c ^ ((nn >> 3) & 1))) = v;
        }
    };

    // ---- this lane's pixel (tile row 2 wave + (lo >> 4), column px_col(lo)) and its 9 halo taps:
    // float offsets of channel quad 2 hi (quad 2 hi + 1 is the same address with bit 4 of the byte
    // offset flipped: the swizzle XORs the quad index)
    const int pr = 2 * wave + (lo >> 4), pc = px_col(lo);
    int toff[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) toff[t] = px_off((pr + t / 3) * HWp + pc + t % 3, 2 * hi);

    floatx16 acc[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[tn][q] = 0.f;

    auto compute = [&](int s, int slot) {
        const int i = s / NK, k0 = (s - i * NK) * BK;
        const float* X = Xs0 + slot * L::XSZ;
        float4 a0 = f4(0.f), a1 = f4(0.f);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const float* kp = taps + t * CIN + k0 + 8 * hi;
            const float4 x0 = *reinterpret_cast<const float4*>(X + toff[t]);
            const float4 x1 = *reinterpret_cast<const float4*>(X + (toff[t] ^ 4));
            a0 = fma4(x0, *reinterpret_cast<const float4*>(kp), a0);
            a1 = fma4(x1, *reinterpret_cast<const float4*>(kp + 4), a1);
        }
        if constexpr (WRITE_Y) {
            int n, h0, w0;
            tile_geom(r + i * G, n, h0, w0);
            float* yp = g.y + ((int64_t)(n * g.H + h0 + pr) * g.W + w0 + pc) * CIN + k0 + 8 * hi;
            st4(yp, a0);
            st4(yp + 4, a1);
        }
        bf16x8 af[3];
        {
            const Split4 s0 = split4(a0), s1 = split4(a1);
            af[0] = __builtin_bit_cast(bf16x8, make_uint4(s0.h.x, s0.h.y, s1.h.x, s1.h.y));
            af[1] = __builtin_bit_cast(bf16x8, make_uint4(s0.m.x, s0.m.y, s1.m.x, s1.m.y));
            af[2] = __builtin_bit_cast(bf16x8, make_uint4(s0.l.x, s0.l.y, s1.l.x, s1.l.y));
        }
        const unsigned short* Bb = reinterpret_cast<const unsigned short*>(smem + L::B0 + slot * L::BSZ);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int nn = tn * 32 + lo;
            const int cs = hi ^ ((nn >> 3) & 1);
            bf16x8 bfr[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bfr[pl] = *reinterpret_cast<const bf16x8*>(Bb + (pl * BN + nn) * BK + 8 * cs);
            acc[tn] = mfma_x6(af, bfr, acc[tn]);
        }
    };

    // ---- statistics: per-wave (mean, M2) of the wave's 32 rows -> red; combined after a barrier
    int pend = -1;  // tile whose per-wave statistics wait in red
    auto combine = [&]() {
        if constexpr (STATS) {
            if (pend >= 0 && wave == (pend & 3)) {
#pragma unroll
                for (int c = lane; c < BN; c += 64) {
                    const float2 s0 = red[c], s1 = red[BN + c], s2 = red[2 * BN + c], s3 = red[3 * BN + c];
                    const float m = ((s0.x + s1.x) + (s2.x + s3.x)) * 0.25f;
                    const float d0 = s0.x - m, d1 = s1.x - m, d2 = s2.x - m, d3 = s3.x - m;
                    const float q = ((s0.y + s1.y) + (s2.y + s3.y)) +
                                    32.f * ((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
                    g.stats[(int64_t)pend * g.Cout + c] = make_float2(m, q);
                }
            }
        }
        pend = -1;
    };
    float* const T = smem + L::T0 + wave * 32 * PTLD;
    auto epilogue = [&](int tile) {
        int n, h0, w0;
        tile_geom(tile, n, h0, w0);
        if constexpr (STATS) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                float sm = 0.f;
#pragma unroll
                for (int q = 0; q < 16; ++q) sm += acc[tn][q];
                sm += __shfl_xor(sm, 32, 64);
                const float m = sm * (1.0f / 32.0f);
                float q2 = 0.f;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const float d = acc[tn][q] - m;
                    q2 = fmaf(d, d, q2);
                }
                q2 += __shfl_xor(q2, 32, 64);
                if (hi == 0) red[wave * BN + tn * 32 + lo] = make_float2(m, q2);
            }
            pend = tile;
        }
        // z (+ the 2x2 pooling selection) through this wave's transpose tile, 32 columns a pass
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
            for (int q = 0; q < 16; ++q) T[acc_row(q, hi) * PTLD + lo] = acc[tn][q];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int cb = tn * 32;
            if (g.zsel) {
                // the wave's two pixel rows hold 8 whole 2x2 windows (T row of pixel (sub, col): col,
                // or 16 + ((col + 2) & 15) on the second row)
                const int j = lane >> 3, qd = lane & 7;  // window j, channel quad qd
                const int c0 = 2 * j, c1 = 2 * j + 1;
                const float4 a = *reinterpret_cast<const float4*>(T + c0 * PTLD + 4 * qd);
                const float4 b = *reinterpret_cast<const float4*>(T + c1 * PTLD + 4 * qd);
                const float4 c = *reinterpret_cast<const float4*>(T + (16 + ((c0 + 2) & 15)) * PTLD + 4 * qd);
                const float4 d = *reinterpret_cast<const float4*>(T + (16 + ((c1 + 2) & 15)) * PTLD + 4 * qd);
                const int col = cb + 4 * qd;
                const unsigned gb = gneg >> (4 * tn);
                float4 o;
                o.x = pool_sel(a.x, b.x, c.x, d.x, (gb & 1u) != 0);
                o.y = pool_sel(a.y, b.y, c.y, d.y, (gb & 2u) != 0);
                o.z = pool_sel(a.z, b.z, c.z, d.z, (gb & 4u) != 0);
                o.w = pool_sel(a.w, b.w, c.w, d.w, (gb & 8u) != 0);
                const int H2 = g.H >> 1, W2 = g.W >> 1;
                st4(g.zsel + ((int64_t)(n * H2 + (h0 >> 1) + wave) * W2 + (w0 >> 1) + j) * g.Cout + col, o);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // 32 pixels x 8 channel quads, 64 per instruction
                const int idx = k * 64 + lane, row = idx >> 3, qd = idx & 7;
                const float4 v = *reinterpret_cast<const float4*>(T + row * PTLD + 4 * qd);
                const int ph = h0 + 2 * wave + (row >> 4), pw = w0 + px_col(row);
                st4(g.z + ((int64_t)(n * g.H + ph) * g.W + pw) * g.Cout + cb + 4 * qd, v);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[tn][q] = 0.f;
    };

    // ---- the stage stream.  Slot s & 1 holds stage s; stage s + 1 was staged (registers -> LDS)
    // at the end of stage s - 1.  Register set t % PD holds stage t from its load until it is staged:
    // when stage s starts, stages s + 1 ... s + PD are in flight (PD = 1: only s + 1).
    using S0 = std::integral_constant<int, 0>;
    if (S > 0) {
        load(0, S0{});
        store(0, 0, S0{});
        if (S > 1) load(1, std::integral_constant<int, 1 % NSET>{});
        if constexpr (PD >= 2) {
            if (S > 2) load(2, std::integral_constant<int, 2 % NSET>{});
        }
        if constexpr (PD >= 3) {
            if (S > 3) load(3, std::integral_constant<int, 3 % NSET>{});
        }
        if constexpr (PD >= 4) {
            if (S > 4) load(4, std::integral_constant<int, 4 % NSET>{});
        }
    }
    __syncthreads();
    auto body = [&](int s, auto cur) {
        // cur: the register set holding stage s + 1, i.e. (s + 1) % PD
        compute(s, s & 1);
        if (s + 1 < S) {
            store(s + 1, (s + 1) & 1, cur);
            if (s + 1 + PD < S) load(s + 1 + PD, cur);
        }
        __syncthreads();
        combine();  // the statistics the waves wrote before this barrier (NK >= 2 stages per tile)
        if (s % NK == NK - 1) epilogue(r + (s / NK) * G);
    };
    for (int s = 0; s < S; s += NSET) {
        body(s, std::integral_constant<int, 1 % NSET>{});
        if constexpr (PD >= 2) {
            if (s + 1 < S) body(s + 1, std::integral_constant<int, 2 % NSET>{});
        }
        if constexpr (PD >= 3) {
            if (s + 2 < S) body(s + 2, std::integral_constant<int, 3 % NSET>{});
        }
        if constexpr (PD >= 4) {
            if (s + 3 < S) body(s + 3, std::integral_constant<int, 4 % NSET>{});
        }
    }
    if constexpr (STATS) {
        __syncthreads();
        combine();
    }
}

template <int MODE, bool DROP, int BN, int CIN, int PD>
void launch_px_t(const SepArgs& a, bool stats, bool write_y, int ntiles, int grid, hipStream_t st) {
#define UNET_PX(ST, WY) sepconv_px_kernel<MODE, DROP, ST, BN, CIN, WY, PD><<<grid, 256, 0, st>>>(a, ntiles)
    if (stats) { if (write_y) UNET_PX(true, true); else UNET_PX(true, false); }
    else { if (write_y) UNET_PX(false, true); else UNET_PX(false, false); }
#undef UNET_PX
}

template <int MODE, bool DROP, int PD>
void launch_px_p(const SepArgs& a, bool stats, bool write_y, int ntiles, int grid, hipStream_t st) {
    if (a.Cout == 64) {
        if (a.Cin == 64) { launch_px_t<MODE, DROP, 64, 64, PD>(a, stats, write_y, ntiles, grid, st); return; }
        launch_px_t<MODE, DROP, 64, 128, PD>(a, stats, write_y, ntiles, grid, st);
    } else {
        if (a.Cin == 64) launch_px_t<MODE, DROP, 128, 64, PD>(a, stats, write_y, ntiles, grid, st);
        else launch_px_t<MODE, DROP, 128, 128, PD>(a, stats, write_y, ntiles, grid, st);
    }
}

template <int MODE, bool DROP>
void launch_px_m(const SepArgs& a, bool stats, bool write_y, int pd, int ntiles, int grid, hipStream_t st) {
#ifdef UNET_LAB_BUILD  // other prefetch depths: lab only (UNET_PX_PD=1, 3, 4)
    if (pd == 1) { launch_px_p<MODE, DROP, 1>(a, stats, write_y, ntiles, grid, st); return; }
    if (pd == 3) { launch_px_p<MODE, DROP, 3>(a, stats, write_y, ntiles, grid, st); return; }
    if (pd == 4) { launch_px_p<MODE, DROP, 4>(a, stats, write_y, ntiles, grid, st); return; }
#endif
    (void)pd;
    launch_px_p<MODE, DROP, 2>(a, stats, write_y, ntiles, grid, st);
}

}  // namespace

bool px_supported(const SepArgs& a, int mode, bool all_shapes) {
    if (!a.pkx || lab_knob("UNET_PX", 1) == 0) return false;  // (lab: UNET_PX=0 keeps the one-tile kernel)
    if (mode != UNET_VIEW_PLAIN && mode != UNET_VIEW_BNRELU && mode != UNET_VIEW_CONCAT) return false;
    if ((a.Cin != 64 && a.Cin != 128) || (a.Cout != 64 && a.Cout != 128)) return false;
    // Only the shapes where it wins INSIDE the train step: 128 outputs from 64 inputs or with the
    // pool-selection epilogue (enc2_block1 79.0 -> 78.2 us, enc2_block2 147.2 -> 138.8 us).  Isolated
    // on a repeated input it also beats the one-tile kernel on 64 -> 64 (1.09-1.14x,
    // profiles/r4l_px_lab.log), but in the step enc1_block2 165 -> 173, dec1_block2 137 -> 158,
    // dec1_block1 258 -> 265, dec2_block2 133 -> 136 us (profiles/r4q_px_in_step.txt).
    // all_shapes (schedule RK) or UNET_PX_ALL=1 (lab) take every supported shape.
    if (!all_shapes && lab_knob("UNET_PX_ALL", 0) == 0 && !(a.Cout == 128 && (a.Cin == 64 || a.zsel))) return false;
    if (mode == UNET_VIEW_CONCAT && a.x.c0 % 16) return false;
    return a.H % TH == 0 && a.W % TW == 0;
}

int launch_px(const SepArgs& a, int mode, bool drop, bool stats, bool write_y, hipStream_t st) {
    if (!px_supported(a, mode, true)) return -1;
    const int ntiles = a.N * (a.H / TH) * (a.W / TW);
    // two blocks per CU; equal runs of tiles (the grid is the tile count / the tiles per block)
    const int slots = 256 * lab_knob("UNET_PX_BPC", 2);
    const int per = (ntiles + slots - 1) / slots;
    const int grid = (ntiles + per - 1) / per;
    const int pd = lab_knob("UNET_PX_PD", 2);
#define UNET_PXM(M) \
    (drop ? launch_px_m<M, true>(a, stats, write_y, pd, ntiles, grid, st) : launch_px_m<M, false>(a, stats, write_y, pd, ntiles, grid, st))
    if (mode == UNET_VIEW_PLAIN) UNET_PXM(UNET_VIEW_PLAIN);
    else if (mode == UNET_VIEW_BNRELU) UNET_PXM(UNET_VIEW_BNRELU);
    else UNET_PXM(UNET_VIEW_CONCAT);
#undef UNET_PXM
    return 0;
}

}  // namespace sep
}  // namespace unet
