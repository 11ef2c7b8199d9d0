// BatchNormalization + ReLU of conv_block (reference model/u_net.py:22-25; Keras 3
// BatchNormalization defaults: momentum 0.99, epsilon 1e-3, batch statistics from
// tf.nn.moments = biased variance, moving stats updated with the same biased variance).
//
// Forward statistics come from the pointwise-GEMM epilogue as per-128-row (mean, M2)
// partials; unet_bn_finalize combines them with Chan's formula in double, in a fixed
// order, and emits the folded affine (scale, shift) that activation views apply on load.
// Backward is two passes over (da, z): per-channel sums (g, g*xhat) then the elementwise
// dz, with the ReLU mask and the consumer's dropout mask recomputed, not stored.
#include "view.h"
#include "lastblock.h"

namespace unet {

namespace {
constexpr int kStatsRows = 128;

// Pass 1: per (chunk of kChunkParts partials, channel) sums of the moments shifted by
// K_c = mean of partial 0 (no cancellation when |mean| >> std):  S1 = sum n_b (mean_b - K),
// S2 = sum M2_b + n_b (mean_b - K)^2, in double, fixed order (4 lanes, then lane order).
// Coalesced: consecutive threads read consecutive channels of one partial row.
constexpr int kChunkParts = 64;
__device__ __forceinline__ void chunk_sums(const float2* __restrict__ part, int64_t nblk, int64_t M, int C, int c,
                                           int lane, int chunk, double& s1, double& s2, float& k_out) {
    const int64_t b0 = (int64_t)chunk * kChunkParts;
    const int64_t b1 = b0 + kChunkParts < nblk ? b0 + kChunkParts : nblk;
    s1 = 0.0;
    s2 = 0.0;
    if (c < C) {
        // every load of the lane (K and its 16 partials) in flight at once: the finish is a chain of
        // dependent round trips on the critical path, so each batch saved is ~1 us per launch
        constexpr int PER = kChunkParts / 4;
        const float2 k0 = part[c];
        float2 pv[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {  // branch-free: a clamped row past the chunk, masked below
            const int64_t b = b0 + lane + 4 * i;
            pv[i] = part[(b < b1 ? b : b0) * C + c];
        }
        k_out = k0.x;
        const double K = (double)k0.x;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int64_t b = b0 + lane + 4 * i;
            if (b < b1) {
                const float2 pm = pv[i];
                const int64_t rows = (M - b * kStatsRows) < kStatsRows ? (M - b * kStatsRows) : kStatsRows;
                const double d = (double)pm.x - K;
                const double nd = (double)rows * d;
                s1 += nd;
                s2 += (double)pm.y + nd * d;
            }
        }
    }
}

__device__ __forceinline__ void bn_apply_channel(int c, float mean, float var, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, float eps, float momentum,
                                                 float* moving_mean, float* moving_var, int update_moving,
                                                 float* mean_out, float* rstd_out, float* scale_out,
                                                 float* shift_out);

// Pass 2 (same launch, lastblock.h): every block publishes its chunk row (sc1 stores); the last
// block of each 64-channel column to arrive sums the rows (4 lanes over interleaved chunks,
// combined in lane order) -> mean, biased var, folded affine, moving update.  One chunk: the
// block's own sums are final.
// the batch (mean, biased var) of channel c -> rstd, the folded affine, the moving update
__device__ __forceinline__ void bn_apply_channel(int c, float mean, float var, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, float eps, float momentum,
                                                 float* moving_mean, float* moving_var, int update_moving,
                                                 float* mean_out, float* rstd_out, float* scale_out,
                                                 float* shift_out) {
    const float rstd = 1.0f / sqrtf(var + eps);
    if (gamma) {
        const float sc = gamma[c] * rstd;
        scale_out[c] = sc;
        shift_out[c] = beta[c] - mean * sc;
    } else {  // use_batch_norm=False: relu(z + bias)
        scale_out[c] = 1.0f;
        shift_out[c] = beta ? beta[c] : 0.f;
    }
    if (mean_out) mean_out[c] = mean;
    if (rstd_out) rstd_out[c] = rstd;
    if (update_moving && moving_mean && moving_var) {
        moving_mean[c] = moving_mean[c] * momentum + mean * (1.0f - momentum);
        moving_var[c] = moving_var[c] * momentum + var * (1.0f - momentum);
    }
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(const float2* __restrict__ part, int64_t nblk, int64_t M,
                                                          int C, double* __restrict__ chunks, unsigned* cnt,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, float momentum,
                                                          float* moving_mean, float* moving_var, int update_moving,
                                                          float* mean_out, float* rstd_out, float* scale_out,
                                                          float* shift_out, double* moments) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int lane = threadIdx.x >> 6;  // = the wave: lane 0 is wave 0, which finalizes
    const int nch = gridDim.y;
    // the finalize's other inputs loaded up front, beside the chunk's partials (its own round trips
    // would otherwise follow the reduction's)
    float gv = 1.f, bv = 0.f, mmv = 0.f, mvv = 0.f;
    if (lane == 0 && c < C && !moments) {
        if (gamma) gv = gamma[c];
        if (beta) bv = beta[c];
        if (update_moving && moving_mean && moving_var) {
            mmv = moving_mean[c];
            mvv = moving_var[c];
        }
    }
    double s1, s2;
    float K = 0.f;  // mean of partial 0 (the shift)
    chunk_sums(part, nblk, M, C, c, lane, blockIdx.y, s1, s2, K);
    __shared__ double r1[256], r2[256];
    __shared__ int flag;
    r1[threadIdx.x] = s1;
    r2[threadIdx.x] = s2;
    __syncthreads();
    if (lane == 0 && c < C)
        for (int l = 1; l < 4; ++l) {
            s1 += r1[threadIdx.x + 64 * l];
            s2 += r2[threadIdx.x + 64 * l];
        }
    if (nch > 1) {
        if (lane == 0 && c < C) {
            st_agent(chunks + ((int64_t)blockIdx.y * C + c) * 2, s1);
            st_agent(chunks + ((int64_t)blockIdx.y * C + c) * 2 + 1, s2);
        }
        if (!last_arrival(cnt + blockIdx.x, (unsigned)nch, &flag)) return;
        s1 = 0.0;
        s2 = 0.0;
        if (c < C) {
            constexpr int FB = 16;  // chunk rows per lane in flight at once (same order of the sums)
            for (int k0 = lane; k0 < nch; k0 += 4 * FB) {
                double a1[FB], a2[FB];
#pragma unroll
                for (int i = 0; i < FB; ++i) {
                    const int k = k0 + 4 * i;
                    a1[i] = k < nch ? ld_agent(chunks + ((int64_t)k * C + c) * 2) : 0.0;
                    a2[i] = k < nch ? ld_agent(chunks + ((int64_t)k * C + c) * 2 + 1) : 0.0;
                }
#pragma unroll
                for (int i = 0; i < FB; ++i)
                    if (k0 + 4 * i < nch) {
                        s1 += a1[i];
                        s2 += a2[i];
                    }
            }
        }
        __syncthreads();  // r1/r2 were read above by lane 0 before the arrival barrier; reuse
        r1[threadIdx.x] = s1;
        r2[threadIdx.x] = s2;
        __syncthreads();
        if (lane == 0 && c < C)
            for (int l = 1; l < 4; ++l) {
                s1 += r1[threadIdx.x + 64 * l];
                s2 += r2[threadIdx.x + 64 * l];
            }
    }
    if (lane != 0 || c >= C) return;
    if (moments) {  // SyncBN: this replica's (count, mean, M2) for the cross-replica combine
        if (c == 0) moments[0] = (double)M;
        moments[1 + c] = (double)K + s1 / (double)M;
        moments[1 + C + c] = s2 - s1 * (s1 / (double)M);
        return;
    }
    const double dm = s1 / (double)M;
    const float mean = (float)((double)K + dm);
    double vd = s2 / (double)M - dm * dm;
    const float var = (float)(vd > 0.0 ? vd : 0.0);
    const float rstd = 1.0f / sqrtf(var + eps);
    if (gamma) {
        const float sc = gv * rstd;
        scale_out[c] = sc;
        shift_out[c] = bv - mean * sc;
    } else {  // use_batch_norm=False: relu(z + bias)
        scale_out[c] = 1.0f;
        shift_out[c] = beta ? bv : 0.f;
    }
    if (mean_out) mean_out[c] = mean;
    if (rstd_out) rstd_out[c] = rstd;
    if (update_moving && moving_mean && moving_var) {
        moving_mean[c] = mmv * momentum + mean * (1.0f - momentum);
        moving_var[c] = mvv * momentum + var * (1.0f - momentum);
    }
}

// SyncBN: the replicas' records [world][1 + 2C] = (count, mean[C], M2[C]) combined in rank order
// (Chan's parallel formula, double; every replica runs the same order on the same gathered records,
// so all end bitwise identical), then the finalize of the global-batch statistics.
__global__ void bn_finalize_moments_kernel(const double* __restrict__ recs, int world, int C,
                                           const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                                           float momentum, float* moving_mean, float* moving_var, int update_moving,
                                           float* mean_out, float* rstd_out, float* scale_out, float* shift_out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int64_t R = 1 + 2 * (int64_t)C;
    double n = recs[0], mu = recs[1 + c], m2 = recs[1 + C + c];
    for (int r = 1; r < world; ++r) {
        const double nr = recs[r * R], mr = recs[r * R + 1 + c], m2r = recs[r * R + 1 + C + c];
        const double nt = n + nr;
        if (nr <= 0.0) continue;
        const double d = mr - mu;
        mu += d * (nr / nt);
        m2 += m2r + d * d * (n * nr / nt);
        n = nt;
    }
    const double vd = m2 / n;
    bn_apply_channel(c, (float)mu, (float)(vd > 0.0 ? vd : 0.0), gamma, beta, eps, momentum, moving_mean, moving_var,
                     update_moving, mean_out, rstd_out, scale_out, shift_out);
}

__global__ void bn_infer_kernel(const float* gamma, const float* beta, const float* mm, const float* mv, int C,
                                float eps, float* scale, float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    if (gamma) {
        const float inv = 1.0f / sqrtf(mv[c] + eps);
        const float sc = gamma[c] * inv;
        scale[c] = sc;
        shift[c] = beta[c] - mm[c] * sc;
    } else {
        scale[c] = 1.0f;
        shift[c] = beta ? beta[c] : 0.f;
    }
}

// Column-block x row-lane geometry shared by the reductions below: CT channel quads per
// block, PL = 256/CT row lanes; rows [chunk * rpc, ...).
struct RedPlan {
    int ctiles, CT;
    int64_t chunks, rpc;
};
RedPlan red_plan(int64_t rows, int cols) {
    RedPlan p;
    const int CQ = cols % 4 == 0 ? cols / 4 : cols;
    p.CT = CQ < 64 ? CQ : 64;
    p.ctiles = (int)cdiv(CQ, p.CT);
    int64_t want = cdiv(1024, p.ctiles);
    int64_t maxc = cdiv(rows, 128);
    p.chunks = want < maxc ? want : maxc;
    if (p.chunks < 1) p.chunks = 1;
    p.rpc = cdiv(rows, p.chunks);
    p.chunks = cdiv(rows, p.rpc);
    return p;
}

// g = da * drop * [z*sc+sh > 0];  partial[chunk][0][c] = sum g, partial[chunk][1][c] = sum g*xhat
template <bool DROP, bool VEC>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ da, const float* __restrict__ z,
                                                            int64_t M, int C, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            float rate, float inv_keep, uint64_t seed, int CT,
                                                            int64_t rpc, float* __restrict__ part,
                                                            unsigned* __restrict__ cnt = nullptr, int ncnt = 0) {
    if (cnt && blockIdx.x == 0 && blockIdx.y == 0)  // the statistics launch that follows counts on them
        for (int i = threadIdx.x; i < ncnt; i += blockDim.x) cnt[i] = 0u;
    const int CQ = VEC ? C / 4 : C;
    const int PL = 256 / CT;
    const int tid = threadIdx.x, cl = tid % CT, pl = tid / CT;
    const int cq = blockIdx.x * CT + cl;
    const int64_t r0 = (int64_t)blockIdx.y * rpc;
    const int64_t r1 = r0 + rpc < M ? r0 + rpc : M;
    __shared__ float4 red[2][256];
    float4 sg = f4(0.f), sgx = f4(0.f);
    if (pl < PL && cq < CQ) {
        if constexpr (VEC) {
            const int c = cq * 4;
            const float4 s4 = ld4(sc + c), h4 = ld4(sh + c), mu = ld4(mean + c), rs = ld4(rstd + c);
            auto accum = [&](int64_t m, float4 zz, float4 g) {
                if constexpr (DROP) {
                    const uint64_t i = (uint64_t)m * C + c;
                    g = mul4(g, drop_mult4(seed, i, rate, inv_keep));
                }
                g.x = fmaf(zz.x, s4.x, h4.x) > 0.f ? g.x : 0.f;
                g.y = fmaf(zz.y, s4.y, h4.y) > 0.f ? g.y : 0.f;
                g.z = fmaf(zz.z, s4.z, h4.z) > 0.f ? g.z : 0.f;
                g.w = fmaf(zz.w, s4.w, h4.w) > 0.f ? g.w : 0.f;
                sg = add4(sg, g);
                const float4 xh = make_float4((zz.x - mu.x) * rs.x, (zz.y - mu.y) * rs.y, (zz.z - mu.z) * rs.z,
                                              (zz.w - mu.w) * rs.w);
                sgx = fma4(g, xh, sgx);
            };
            int64_t m = r0 + pl;
            for (; m + 3 * PL < r1; m += 4 * PL) {  // 8 loads in flight per thread
                float4 zz[4], dd[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    zz[u] = ld4(z + (m + u * PL) * C + c);
                    dd[u] = ld4(da + (m + u * PL) * C + c);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) accum(m + u * PL, zz[u], dd[u]);
            }
            for (; m < r1; m += PL) accum(m, ld4(z + m * C + c), ld4(da + m * C + c));
        } else {
            const int c = cq;
            const float s1 = sc[c], h1 = sh[c], mu = mean[c], rs = rstd[c];
            for (int64_t m = r0 + pl; m < r1; m += PL) {
                const float zz = z[m * C + c];
                float g = da[m * C + c];
                if constexpr (DROP) g *= drop_mult(seed, (uint64_t)m * C + c, rate, inv_keep);
                g = fmaf(zz, s1, h1) > 0.f ? g : 0.f;
                sg.x += g;
                sgx.x = fmaf(g, (zz - mu) * rs, sgx.x);
            }
        }
    }
    red[0][tid] = sg;
    red[1][tid] = sgx;
    __syncthreads();
    if (pl == 0 && cq < CQ) {
        float4 a = red[0][cl], b = red[1][cl];
        for (int q = 1; q < PL; ++q) {
            a = add4(a, red[0][q * CT + cl]);
            b = add4(b, red[1][q * CT + cl]);
        }
        float* out = part + (int64_t)blockIdx.y * 2 * C;
        if constexpr (VEC) {
            st4(out + cq * 4, a);
            st4(out + C + cq * 4, b);
        } else {
            out[cq] = a.x;
            out[C + cq] = b.x;
        }
    }
}

template <bool DROP, bool VEC>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ da, const float* __restrict__ z,
                                                           int64_t M, int C, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ sc, const float* __restrict__ sh,
                                                           float rate, float inv_keep, uint64_t seed, int use_bn,
                                                           const float* __restrict__ sums, float* __restrict__ dz) {
    const int CQ = VEC ? C / 4 : C;
    const int64_t total = M * CQ;
    const float invM = 1.0f / (float)M;
    for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int cq = (int)(idx % CQ);
        const int64_t m = idx / CQ;
        if constexpr (VEC) {
            const int c = cq * 4;
            const float4 zz = ld4(z + m * C + c), s4 = ld4(sc + c), h4 = ld4(sh + c);
            float4 g = ld4(da + m * C + c);
            if constexpr (DROP) {
                const uint64_t i = (uint64_t)m * C + c;
                g = mul4(g, drop_mult4(seed, i, rate, inv_keep));
            }
            g.x = fmaf(zz.x, s4.x, h4.x) > 0.f ? g.x : 0.f;
            g.y = fmaf(zz.y, s4.y, h4.y) > 0.f ? g.y : 0.f;
            g.z = fmaf(zz.z, s4.z, h4.z) > 0.f ? g.z : 0.f;
            g.w = fmaf(zz.w, s4.w, h4.w) > 0.f ? g.w : 0.f;
            float4 o = g;
            if (use_bn) {
                const float4 mu = ld4(mean + c), rs = ld4(rstd + c);
                const float4 sb = ld4(sums + c), sgx = ld4(sums + C + c);
                o.x = s4.x * (g.x - sb.x * invM - (zz.x - mu.x) * rs.x * sgx.x * invM);
                o.y = s4.y * (g.y - sb.y * invM - (zz.y - mu.y) * rs.y * sgx.y * invM);
                o.z = s4.z * (g.z - sb.z * invM - (zz.z - mu.z) * rs.z * sgx.z * invM);
                o.w = s4.w * (g.w - sb.w * invM - (zz.w - mu.w) * rs.w * sgx.w * invM);
            }
            st4(dz + m * C + c, o);
        } else {
            const int c = cq;
            const float zz = z[m * C + c];
            float g = da[m * C + c];
            if constexpr (DROP) g *= drop_mult(seed, (uint64_t)m * C + c, rate, inv_keep);
            g = fmaf(zz, sc[c], sh[c]) > 0.f ? g : 0.f;
            float o = g;
            if (use_bn) o = sc[c] * (g - sums[c] * invM - (zz - mean[c]) * rstd[c] * sums[C + c] * invM);
            dz[m * C + c] = o;
        }
    }
}

// scatter the reduced sums: dbeta = sums[0], dgamma = sums[1]
__global__ void bn_bwd_store_kernel(const float* sums, int C, int use_bn, float* dgamma, float* dbeta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    if (dbeta) dbeta[c] = sums[c];
    if (use_bn && dgamma) dgamma[c] = sums[C + c];
}

// dbeta = S1, dgamma = S2 and the dz coefficients of A_BNBWD loads (gemm.hip):
// coef = (mu, p, q) with p = S1 / M, q = rstd * S2 / M (zeros without BatchNorm: dz = g).
__global__ void bn_bwd_coef_kernel(const float* sums, int C, int64_t M, int use_bn, const float* mean,
                                   const float* rstd, float* dgamma, float* dbeta, float* coef) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float s1 = sums[c], s2 = sums[C + c];
    if (dbeta) dbeta[c] = s1;
    if (use_bn && dgamma) dgamma[c] = s2;
    const float invM = 1.0f / (float)M;
    coef[c] = use_bn ? mean[c] : 0.f;
    coef[C + c] = use_bn ? s1 * invM : 0.f;
    coef[2 * C + c] = use_bn ? rstd[c] * (s2 * invM) : 0.f;
}

// Statistics-only finish: the fixed-order slab reduction of (S1, S2) fused with the coefficient
// kernel above, in ONE launch.  Block (x, y) = 16 channel quads x 16 slab groups over slabs
// [64 y, 64 y + 64) (all S slabs when the grid has one row); groups are combined by wave shuffles
// and a 4-wave LDS step (4 KB of LDS: the block still fits beside side-stream GEMM blocks that
// hold most of a CU's LDS -- the 32 KB version waited up to 140 us for a slot, r1zd).  With
// several rows each block publishes its chunk row (double) and the last block of column x to
// arrive (lastblock.h) sums the rows in order and writes dgamma / dbeta / coef.
constexpr int kLQ = 16, kSG = 16;
__device__ __forceinline__ void group_reduce8(double* a, double (*red)[8][kLQ]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] += __shfl_xor(a[k], 16);
        a[k] += __shfl_xor(a[k], 32);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane < kLQ) {
#pragma unroll
        for (int k = 0; k < 8; ++k) red[w][k][lane] = a[k];
    }
    __syncthreads();
    if (threadIdx.x < kLQ) {
        const int t = threadIdx.x;
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = ((red[0][k][t] + red[1][k][t]) + red[2][k][t]) + red[3][k][t];
    }
}
__global__ __launch_bounds__(256) void bn_bwd_stats_kernel(const float* __restrict__ part, int S, int C, int64_t M,
                                                           int use_bn, const float* mean, const float* rstd,
                                                           float* dgamma, float* dbeta, float* coef,
                                                           double* chunks, unsigned* cnt) {
    main_stream_prio();
    const int q = threadIdx.x % kLQ, g = threadIdx.x / kLQ;
    const int c = (blockIdx.x * kLQ + q) * 4;
    const int nch = gridDim.y;
    const int s0 = blockIdx.y * kGroupSlabs, s1 = nch == 1 || s0 + kGroupSlabs > S ? S : s0 + kGroupSlabs;
    __shared__ double red[4][8][kLQ];
    __shared__ int flag;
    // the writers' mean / rstd loaded up front: loaded after the first output store they would each
    // wait for it (the pointers may alias), a chain of 8 round trips at the end of the launch
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, rs[4] = {0.f, 0.f, 0.f, 0.f};
    if (threadIdx.x < kLQ && c < C && use_bn) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            mu[k] = mean[c + k];
            rs[k] = rstd[c + k];
        }
    }
    double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (c < C) {
        int s = s0 + g;
        for (; s + 3 * kSG < s1; s += 4 * kSG) {  // 8 loads in flight
            float4 u[4], v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u[k] = ld4(part + (int64_t)(s + k * kSG) * 2 * C + c);
                v[k] = ld4(part + (int64_t)(s + k * kSG) * 2 * C + C + c);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a[0] += (double)u[k].x; a[1] += (double)u[k].y; a[2] += (double)u[k].z; a[3] += (double)u[k].w;
                a[4] += (double)v[k].x; a[5] += (double)v[k].y; a[6] += (double)v[k].z; a[7] += (double)v[k].w;
            }
        }
        for (; s < s1; s += kSG) {
            const float4 u = ld4(part + (int64_t)s * 2 * C + c), v = ld4(part + (int64_t)s * 2 * C + C + c);
            a[0] += (double)u.x; a[1] += (double)u.y; a[2] += (double)u.z; a[3] += (double)u.w;
            a[4] += (double)v.x; a[5] += (double)v.y; a[6] += (double)v.z; a[7] += (double)v.w;
        }
    }
    group_reduce8(a, red);
    if (nch > 1) {
        if (threadIdx.x < kLQ && c < C) {
            double* row = chunks + (int64_t)blockIdx.y * 2 * C;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                st_agent(row + c + k, a[k]);
                st_agent(row + C + c + k, a[4 + k]);
            }
        }
        if (!last_arrival(cnt + blockIdx.x, (unsigned)nch, &flag)) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = 0.0;
        if (c < C) {
            int r = g;
            for (; r + kSG < nch; r += 2 * kSG) {
                double u[2][8];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        u[h][k] = ld_agent(chunks + (int64_t)(r + h * kSG) * 2 * C + c + k);
                        u[h][4 + k] = ld_agent(chunks + (int64_t)(r + h * kSG) * 2 * C + C + c + k);
                    }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int k = 0; k < 8; ++k) a[k] += u[h][k];
            }
            for (; r < nch; r += kSG)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    a[k] += ld_agent(chunks + (int64_t)r * 2 * C + c + k);
                    a[4 + k] += ld_agent(chunks + (int64_t)r * 2 * C + C + c + k);
                }
        }
        group_reduce8(a, red);
    }
    if (threadIdx.x >= kLQ || c >= C) return;
    const float invM = 1.0f / (float)M;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int cc = c + k;
        const float s1v = (float)a[k], s2v = (float)a[4 + k];
        if (dbeta) dbeta[cc] = s1v;
        if (use_bn && dgamma) dgamma[cc] = s2v;
        coef[cc] = use_bn ? mu[k] : 0.f;
        coef[C + cc] = use_bn ? s1v * invM : 0.f;
        coef[2 * C + cc] = use_bn ? rs[k] * (s2v * invM) : 0.f;
    }
}

// dgamma / dbeta / coef from S slabs [S][2c] (c % 4 == 0) in one launch; with more than 64 slabs
// it needs `scratch` (cdiv(S, 64) x 2c doubles) and cdiv(c, 64) counters that are zero on entry
// (left zero on exit).
int bwd_stats_finish(const float* part, int S, int c, int64_t m, int use_bn, const float* mean, const float* rstd,
                     float* dgamma, float* dbeta, float* coef, double* scratch, unsigned* cnt, hipStream_t st) {
    if (lab_knob("UNET_SKIP_BNBWD", 0)) return 0;  // lab: upper bound of folding the launch away
    const unsigned gx = (unsigned)cdiv(c / 4, kLQ);
    const unsigned nch = S <= kGroupSlabs ? 1u : (unsigned)cdiv(S, kGroupSlabs);
    bn_bwd_stats_kernel<<<dim3(gx, nch), 256, 0, st>>>(part, S, c, m, use_bn, mean, rstd, dgamma, dbeta, coef, scratch,
                                                       cnt);
    UNET_CHECK_LAUNCH("bn backward statistics (finish)");
    return 0;
}

template <bool VEC>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ x, int64_t rows, int C, int CT,
                                                     int64_t rpc, float* __restrict__ part) {
    const int CQ = VEC ? C / 4 : C;
    const int PL = 256 / CT;
    const int tid = threadIdx.x, cl = tid % CT, pl = tid / CT;
    const int cq = blockIdx.x * CT + cl;
    const int64_t r0 = (int64_t)blockIdx.y * rpc;
    const int64_t r1 = r0 + rpc < rows ? r0 + rpc : rows;
    __shared__ float4 red[256];
    float4 s = f4(0.f);
    if (pl < PL && cq < CQ) {
        if constexpr (VEC) {
            for (int64_t m = r0 + pl; m < r1; m += PL) s = add4(s, ld4(x + m * C + cq * 4));
        } else {
            for (int64_t m = r0 + pl; m < r1; m += PL) s.x += x[m * C + cq];
        }
    }
    red[tid] = s;
    __syncthreads();
    if (pl == 0 && cq < CQ) {
        float4 a = red[cl];
        for (int q = 1; q < PL; ++q) a = add4(a, red[q * CT + cl]);
        float* out = part + (int64_t)blockIdx.y * C;
        if constexpr (VEC)
            st4(out + cq * 4, a);
        else
            out[cq] = a.x;
    }
}

int grid_for(int64_t work) {
    int64_t g = cdiv(work, 256);
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (int)g;
}
}  // namespace

size_t bn_partials_bytes(int64_t m, int c);
size_t colsum_workspace(int64_t rows, int cols) {
    RedPlan p = red_plan(rows, cols);
    return align_up((size_t)p.chunks * cols * sizeof(float), 256);
}

int colsum(const float* x, int64_t rows, int cols, float* out, void* ws, size_t ws_bytes, hipStream_t st) {
    RedPlan p = red_plan(rows, cols);
    const size_t need = (size_t)p.chunks * cols * sizeof(float);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "colsum: workspace %zu < %zu", ws_bytes, need);
    float* part = static_cast<float*>(ws);
    dim3 grid(p.ctiles, (unsigned)p.chunks);
    if (cols % 4 == 0)
        colsum_kernel<true><<<grid, 256, 0, st>>>(x, rows, cols, p.CT, p.rpc, part);
    else
        colsum_kernel<false><<<grid, 256, 0, st>>>(x, rows, cols, p.CT, p.rpc, part);
    UNET_CHECK_LAUNCH("colsum");
    return reduce_slabs(part, (int)p.chunks, cols, out, cols, cols, st);
}

}  // namespace unet

using namespace unet;

size_t unet::bn_partials_bytes(int64_t m, int c) {
    const int64_t nblk = cdiv(m, kStatsRows);
    return align_up((size_t)nblk * c * sizeof(float2), 256) +  // per-tile partials
           align_up((size_t)cdiv(nblk, kChunkParts) * c * sizeof(double2), 256) +  // chunk rows
           (size_t)cdiv(c, 64) * sizeof(unsigned);  // finalize arrival counters (zero at allocation)
}

extern "C" int unet_bn_finalize(float* bn_partials, int64_t m, int c, const float* gamma, const float* beta,
                                float eps, float momentum, float* moving_mean, float* moving_var, int update_moving,
                                float* mean, float* rstd, float* scale, float* shift, unet_stream_t stream) {
    UNET_CHECK_ARG(bn_partials && scale && shift && m > 0 && c > 0, "unet_bn_finalize: bad args");
    UNET_CHECK_ARG(!gamma || beta, "unet_bn_finalize: gamma without beta");
    hipStream_t st = as_stream(stream);
    if (lab_knob("UNET_SKIP_BNFIN", 0)) return 0;  // lab: upper bound of folding the launch away
    const int64_t nblk = cdiv(m, kStatsRows);
    const int nch = (int)cdiv(nblk, kChunkParts);
    const float2* part = reinterpret_cast<const float2*>(bn_partials);
    double* chunks = reinterpret_cast<double*>(reinterpret_cast<char*>(bn_partials) +
                                               align_up((size_t)nblk * c * sizeof(float2), 256));
    unsigned* cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(bn_partials) +
                                                align_up((size_t)nblk * c * sizeof(float2), 256) +
                                                align_up((size_t)nch * c * sizeof(double2), 256));
    bn_finalize_kernel<<<dim3((unsigned)cdiv(c, 64), (unsigned)nch), 256, 0, st>>>(
        part, nblk, m, c, chunks, cnt, gamma, beta, eps, momentum, moving_mean, moving_var, update_moving, mean, rstd,
        scale, shift, nullptr);
    UNET_CHECK_LAUNCH("unet_bn_finalize");
    return 0;
}

extern "C" int unet_bn_moments(float* bn_partials, int64_t m, int c, double* moments, unet_stream_t stream) {
    UNET_CHECK_ARG(bn_partials && moments && m > 0 && c > 0, "unet_bn_moments: bad args");
    const int64_t nblk = cdiv(m, kStatsRows);
    const int nch = (int)cdiv(nblk, kChunkParts);
    const float2* part = reinterpret_cast<const float2*>(bn_partials);
    double* chunks = reinterpret_cast<double*>(reinterpret_cast<char*>(bn_partials) +
                                               align_up((size_t)nblk * c * sizeof(float2), 256));
    unsigned* cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(bn_partials) +
                                                align_up((size_t)nblk * c * sizeof(float2), 256) +
                                                align_up((size_t)nch * c * sizeof(double2), 256));
    bn_finalize_kernel<<<dim3((unsigned)cdiv(c, 64), (unsigned)nch), 256, 0, as_stream(stream)>>>(
        part, nblk, m, c, chunks, cnt, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
        nullptr, moments);
    UNET_CHECK_LAUNCH("unet_bn_moments");
    return 0;
}

extern "C" int unet_bn_finalize_moments(const double* moments, int world, int c, const float* gamma,
                                        const float* beta, float eps, float momentum, float* moving_mean,
                                        float* moving_var, int update_moving, float* mean, float* rstd, float* scale,
                                        float* shift, unet_stream_t stream) {
    UNET_CHECK_ARG(moments && world > 0 && c > 0 && scale && shift, "unet_bn_finalize_moments: bad args");
    UNET_CHECK_ARG(!gamma || beta, "unet_bn_finalize_moments: gamma without beta");
    bn_finalize_moments_kernel<<<(unsigned)cdiv(c, 256), 256, 0, as_stream(stream)>>>(
        moments, world, c, gamma, beta, eps, momentum, moving_mean, moving_var, update_moving, mean, rstd, scale,
        shift);
    UNET_CHECK_LAUNCH("unet_bn_finalize_moments");
    return 0;
}

extern "C" int unet_bn_bwd_coef(const float* sums, int64_t m, int c, int use_bn, const float* mean,
                                const float* rstd, float* coef, unet_stream_t stream) {
    UNET_CHECK_ARG(sums && coef && m > 0 && c > 0, "unet_bn_bwd_coef: bad args");
    UNET_CHECK_ARG(!use_bn || (mean && rstd), "unet_bn_bwd_coef: use_bn needs mean/rstd");
    bn_bwd_coef_kernel<<<(unsigned)cdiv(c, 256), 256, 0, as_stream(stream)>>>(sums, c, m, use_bn, mean, rstd, nullptr,
                                                                               nullptr, coef);
    UNET_CHECK_LAUNCH("unet_bn_bwd_coef");
    return 0;
}

extern "C" int unet_bn_infer_params(const float* gamma, const float* beta, const float* moving_mean,
                                    const float* moving_var, int c, float eps, float* scale, float* shift,
                                    unet_stream_t stream) {
    UNET_CHECK_ARG(scale && shift && c > 0, "unet_bn_infer_params: bad args");
    UNET_CHECK_ARG(!gamma || (beta && moving_mean && moving_var), "unet_bn_infer_params: missing BN tensors");
    bn_infer_kernel<<<(unsigned)cdiv(c, 256), 256, 0, as_stream(stream)>>>(gamma, beta, moving_mean, moving_var, c,
                                                                           eps, scale, shift);
    UNET_CHECK_LAUNCH("unet_bn_infer_params");
    return 0;
}

extern "C" size_t unet_bn_relu_bwd_workspace(int64_t m, int c) {
    if (m <= 0 || c <= 0) return 0;
    RedPlan p = red_plan(m, c);
    return align_up((size_t)p.chunks * 2 * c * sizeof(float), 256) + align_up((size_t)2 * c * sizeof(float), 256) +
           align_up((size_t)cdiv(p.chunks, kGroupSlabs) * 2 * c * sizeof(double), 256) +  // finish scratch
           align_up((size_t)cdiv(c, 64) * sizeof(unsigned), 256);  // finish counters (zeroed by the reduce launch)
}

namespace {
int bn_relu_bwd_impl(const float* da, const float* z, int64_t m, int c, const float* mean, const float* rstd,
                     const float* scale, const float* shift, int use_bn, float drop_rate, uint64_t drop_seed,
                     float* dgamma, float* dbeta, float* dz, float* coef_out, void* ws, size_t ws_bytes,
                     unet_stream_t stream) {
    UNET_CHECK_ARG(da && z && scale && shift && (dz || coef_out) && m > 0 && c > 0, "unet_bn_relu_bwd: bad args");
    UNET_CHECK_ARG(!use_bn || (mean && rstd), "unet_bn_relu_bwd: use_bn needs mean/rstd");
    UNET_CHECK_ARG(drop_rate >= 0.f && drop_rate < 1.f, "unet_bn_relu_bwd: bad drop_rate");
    const size_t need = unet_bn_relu_bwd_workspace(m, c);
    UNET_CHECK_ARG(ws && ws_bytes >= need, "unet_bn_relu_bwd: workspace %zu < %zu", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    RedPlan p = red_plan(m, c);
    float* part = static_cast<float*>(ws);
    float* sums = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                           align_up((size_t)p.chunks * 2 * c * sizeof(float), 256));
    const float* mu = use_bn ? mean : scale;  // unused when !use_bn (mask only)
    const float* rs = use_bn ? rstd : scale;
    const float inv_keep = drop_rate > 0.f ? 1.0f / (1.0f - drop_rate) : 1.0f;
    const bool vec = c % 4 == 0;
    const bool drop = drop_rate > 0.f;
    const bool stats_only = coef_out && vec;  // reduce + one statistics launch (bwd_stats_finish)
    double* scratch = reinterpret_cast<double*>(reinterpret_cast<char*>(sums) +
                                                align_up((size_t)2 * c * sizeof(float), 256));
    unsigned* cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(scratch) +
                                                align_up((size_t)cdiv(p.chunks, kGroupSlabs) * 2 * c * sizeof(double), 256));
    const int ncnt = stats_only ? (int)cdiv(c, 64) : 0;
    dim3 grid(p.ctiles, (unsigned)p.chunks);
#define UNET_BNB(D, V)                                                                                        \
    bn_bwd_reduce_kernel<D, V><<<grid, 256, 0, st>>>(da, z, m, c, mu, rs, scale, shift, drop_rate, inv_keep, \
                                                     drop_seed, p.CT, p.rpc, part, ncnt ? cnt : nullptr, ncnt)
    if (drop) {
        if (vec) UNET_BNB(true, true);
        else UNET_BNB(true, false);
    } else {
        if (vec) UNET_BNB(false, true);
        else UNET_BNB(false, false);
    }
#undef UNET_BNB
    UNET_CHECK_LAUNCH("unet_bn_relu_bwd(reduce)");
    if (stats_only)  // statistics-only entry (unet_bn_relu_bwd_stats): reduce + coefficients
        return bwd_stats_finish(part, (int)p.chunks, c, m, use_bn, mean, rstd, dgamma, dbeta, coef_out, scratch, cnt,
                                st);
    int rc = reduce_slabs(part, (int)p.chunks, (int64_t)2 * c, sums, (int64_t)2 * c, (int64_t)2 * c, st);
    if (rc) return rc;
    if (coef_out) {  // statistics-only entry (unet_bn_relu_bwd_stats): no dz pass
        bn_bwd_coef_kernel<<<(unsigned)cdiv(c, 256), 256, 0, st>>>(sums, c, m, use_bn, mean, rstd, dgamma, dbeta,
                                                                    coef_out);
        UNET_CHECK_LAUNCH("unet_bn_relu_bwd_stats(coef)");
        return 0;
    }
    bn_bwd_store_kernel<<<(unsigned)cdiv(c, 256), 256, 0, st>>>(sums, c, use_bn, dgamma, dbeta);
    UNET_CHECK_LAUNCH("unet_bn_relu_bwd(store)");
    const int64_t work = m * (vec ? c / 4 : c);
    const int g2 = grid_for(work);
#define UNET_BNA(D, V)                                                                                             \
    bn_bwd_apply_kernel<D, V><<<g2, 256, 0, st>>>(da, z, m, c, mu, rs, scale, shift, drop_rate, inv_keep, drop_seed, \
                                                  use_bn, sums, dz)
    if (drop) {
        if (vec) UNET_BNA(true, true);
        else UNET_BNA(true, false);
    } else {
        if (vec) UNET_BNA(false, true);
        else UNET_BNA(false, false);
    }
#undef UNET_BNA
    UNET_CHECK_LAUNCH("unet_bn_relu_bwd(apply)");
    return 0;
}
}  // namespace

extern "C" int unet_bn_relu_bwd(const float* da, const float* z, int64_t m, int c, const float* mean,
                                const float* rstd, const float* scale, const float* shift, int use_bn,
                                float drop_rate, uint64_t drop_seed, float* dgamma, float* dbeta, float* dz,
                                void* ws, size_t ws_bytes, unet_stream_t stream) {
    UNET_CHECK_ARG(dz, "unet_bn_relu_bwd: null dz");
    return bn_relu_bwd_impl(da, z, m, c, mean, rstd, scale, shift, use_bn, drop_rate, drop_seed, dgamma, dbeta, dz,
                            nullptr, ws, ws_bytes, stream);
}

extern "C" size_t unet_bn_stats_partials_size(int S, int c) {
    if (S <= 0 || c <= 0) return 0;
    return bnpart_bytes(S, c);  // slabs | double scratch | in-launch finish counters (lastblock.h)
}

extern "C" int unet_bn_relu_bwd_stats_finish(float* partials, int S, int64_t m, int c, const float* mean,
                                             const float* rstd, int use_bn, float* dgamma, float* dbeta, float* coef,
                                             unet_stream_t stream) {
    UNET_CHECK_ARG(partials && coef && S > 0 && m > 0 && c > 0, "unet_bn_relu_bwd_stats_finish: bad args");
    UNET_CHECK_ARG(c % 4 == 0, "unet_bn_relu_bwd_stats_finish: channels must be a multiple of 4");
    UNET_CHECK_ARG(!use_bn || (mean && rstd), "unet_bn_relu_bwd_stats_finish: use_bn needs mean/rstd");
    double* scratch = reinterpret_cast<double*>(reinterpret_cast<char*>(partials) + bnpart_scratch_off(S, c));
    unsigned* cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(partials) + bnpart_counter_off(S, c));
    return bwd_stats_finish(partials, S, c, m, use_bn, mean, rstd, dgamma, dbeta, coef, scratch, cnt,
                            as_stream(stream));
}

extern "C" int unet_bn_relu_bwd_stats(const float* da, const float* z, int64_t m, int c, const float* mean,
                                      const float* rstd, const float* scale, const float* shift, int use_bn,
                                      float drop_rate, uint64_t drop_seed, float* dgamma, float* dbeta, float* coef,
                                      void* ws, size_t ws_bytes, unet_stream_t stream) {
    UNET_CHECK_ARG(coef, "unet_bn_relu_bwd_stats: null coef");
    return bn_relu_bwd_impl(da, z, m, c, mean, rstd, scale, shift, use_bn, drop_rate, drop_seed, dgamma, dbeta,
                            nullptr, coef, ws, ws_bytes, stream);
}
