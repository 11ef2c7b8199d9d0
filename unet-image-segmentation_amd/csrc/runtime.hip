// Error reporting, view validation and the deterministic slab reduction shared by
// every op of libunet_hip.so.
#include <stdarg.h>

#include "view.h"

namespace unet {

namespace {
thread_local char g_err[512] = "";

__device__ __forceinline__ void store_out(float* out, int64_t l, int64_t row, int64_t ld_out, double v) {
    out[(l / row) * ld_out + (l % row)] = (float)v;
}

// out[l] = sum_s part[s][l] with s in increasing order, in double.  Wide reductions (many
// outputs): one thread per 4 consecutive outputs walks all S slabs with float4 loads.
__global__ __launch_bounds__(256) void reduce_cols4_kernel(const float* __restrict__ part, int S, int64_t L, int64_t sp,
                                                           float* __restrict__ out, int64_t row, int64_t ld_out) {
    const int64_t l = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (l >= L) return;
    const float* p = part + l;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int s = 0;
    for (; s + 4 <= S; s += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ld4(p + (int64_t)(s + u) * sp);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a0 += (double)v[u].x;
            a1 += (double)v[u].y;
            a2 += (double)v[u].z;
            a3 += (double)v[u].w;
        }
    }
    for (; s < S; ++s) {
        const float4 v = ld4(p + (int64_t)s * sp);
        a0 += (double)v.x;
        a1 += (double)v.y;
        a2 += (double)v.z;
        a3 += (double)v.w;
    }
    store_out(out, l, row, ld_out, a0);
    store_out(out, l + 1, row, ld_out, a1);
    store_out(out, l + 2, row, ld_out, a2);
    store_out(out, l + 3, row, ld_out, a3);
}

// Grouped reductions: block = (512/G) output quads x G slab groups; group g sums slabs g, g+G, ...
// in increasing order (4 loads in flight), then a fixed-order tree adds the G group partials.  G
// is picked so that enough loads are in flight chip-wide (few outputs -> more groups).
template <int G>
__global__ __launch_bounds__(512) void reduce_grp4_kernel(const float* __restrict__ part, int S, int64_t L, int64_t sp,
                                                          float* __restrict__ out, int64_t row, int64_t ld_out) {
    constexpr int LQ = 512 / G;
    const int q = threadIdx.x % LQ, g = threadIdx.x / LQ;
    const int64_t l = ((int64_t)blockIdx.x * LQ + q) * 4;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    if (l < L) {
        int s = g;
        for (; s + 3 * G < S; s += 4 * G) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = ld4(part + (int64_t)(s + u * G) * sp + l);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a[0] += (double)v[u].x; a[1] += (double)v[u].y; a[2] += (double)v[u].z; a[3] += (double)v[u].w;
            }
        }
        for (; s < S; s += G) {
            const float4 v0 = ld4(part + (int64_t)s * sp + l);
            a[0] += (double)v0.x; a[1] += (double)v0.y; a[2] += (double)v0.z; a[3] += (double)v0.w;
        }
    }
    __shared__ double red[4][512];
#pragma unroll
    for (int k = 0; k < 4; ++k) red[k][threadIdx.x] = a[k];
    __syncthreads();
    for (int half = G / 2; half > 0; half >>= 1) {
        if (g < half) {
#pragma unroll
            for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + half * LQ];
        }
        __syncthreads();
    }
    if (g == 0 && l < L) {
#pragma unroll
        for (int k = 0; k < 4; ++k) store_out(out, l + k, row, ld_out, red[k][q]);
    }
}
// In-place first level for long, narrow reductions (few outputs, many slabs: the single pass would
// run on a handful of blocks, each walking thousands of slabs): chunk c of CH consecutive slabs is
// summed (fixed order, double) into its first slab, c * CH, which only this chunk reads.  The
// second level then reduces the chunk leaders (slab pitch CH * sp).
__global__ __launch_bounds__(256) void reduce_chunk_kernel(float* __restrict__ part, int S, int64_t L, int64_t sp, int CH) {
    const int64_t l = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    const int s0 = blockIdx.y * CH, s1 = s0 + CH < S ? s0 + CH : S;
    if (l >= L) return;
    float* p = part + (int64_t)s0 * sp + l;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ld4(p + (int64_t)(s - s0 + u) * sp);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a0 += (double)v[u].x;
            a1 += (double)v[u].y;
            a2 += (double)v[u].z;
            a3 += (double)v[u].w;
        }
    }
    for (; s < s1; ++s) {
        const float4 v = ld4(p + (int64_t)(s - s0) * sp);
        a0 += (double)v.x;
        a1 += (double)v.y;
        a2 += (double)v.z;
        a3 += (double)v.w;
    }
    st4(p, make_float4((float)a0, (float)a1, (float)a2, (float)a3));
}
// One output (L == 1: S contiguous values, e.g. the head's bias gradient partials): 1024 threads
// stride over the values in double, then a fixed-order LDS tree.
__global__ __launch_bounds__(1024) void reduce_one_kernel(const float* __restrict__ part, int S, float* __restrict__ out,
                                                          int64_t row, int64_t ld_out) {
    double a = 0.0;
    for (int s = threadIdx.x; s < S; s += 1024) a += (double)part[s];
    __shared__ double red[1024];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int h = 512; h > 0; h >>= 1) {
        if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) store_out(out, 0, row, ld_out, red[0]);
}
// Scalar fallback for L % 4 != 0: block = 64 outputs x 16 slab groups.
__global__ __launch_bounds__(1024) void reduce_slabs_kernel(const float* __restrict__ part, int S, int64_t L, int64_t sp,
                                                            float* __restrict__ out, int64_t row, int64_t ld_out) {
    constexpr int G = 16;
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t l = (int64_t)blockIdx.x * 64 + lane;
    double acc = 0.0;
    if (l < L)
        for (int s = g; s < S; s += G) acc += (double)part[(int64_t)s * sp + l];
    __shared__ double red[G][64];
    red[g][lane] = acc;
    __syncthreads();
    if (g == 0 && l < L) {
        double t = red[0][lane];
        for (int k = 1; k < G; ++k) t += red[k][lane];
        store_out(out, l, row, ld_out, t);
    }
}
// reduce_slabs_pair: blocks [0, a.nblk) reduce array a, the rest array b (block-uniform), each
// thread 4 consecutive outputs over slabs g, g + 32, ... in increasing order (4 loads in flight;
// float4 when the array is 16-B aligned with L % 4 == 0, guarded scalars otherwise), then the
// fixed-order tree of reduce_grp4_kernel<32> -- for a float4 array the same sums, bit for bit.
struct SlabArr {
    const float* part;
    int64_t L;
    float* out;
    int nblk;
    int vec;
};
__global__ __launch_bounds__(512) void reduce_pair_kernel(SlabArr a, SlabArr b, int S) {
    constexpr int G = 32, LQ = 512 / G;
    const bool second = (int)blockIdx.x >= a.nblk;
    const float* part = second ? b.part : a.part;
    const int64_t L = second ? b.L : a.L;
    float* out = second ? b.out : a.out;
    const int vec = second ? b.vec : a.vec;
    const int bx = second ? (int)blockIdx.x - a.nblk : (int)blockIdx.x;
    const int q = threadIdx.x % LQ, g = threadIdx.x / LQ;
    const int64_t l = ((int64_t)bx * LQ + q) * 4;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (l < L) {
        int s = g;
        if (vec) {
            for (; s + 3 * G < S; s += 4 * G) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = ld4(part + (int64_t)(s + u * G) * L + l);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc[0] += (double)v[u].x; acc[1] += (double)v[u].y; acc[2] += (double)v[u].z; acc[3] += (double)v[u].w;
                }
            }
            for (; s < S; s += G) {
                const float4 v0 = ld4(part + (int64_t)s * L + l);
                acc[0] += (double)v0.x; acc[1] += (double)v0.y; acc[2] += (double)v0.z; acc[3] += (double)v0.w;
            }
        } else {
            const int nk = L - l < 4 ? (int)(L - l) : 4;
            for (; s + 3 * G < S; s += 4 * G) {  // 4 slabs' loads in flight
                float v[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {  // clamped, unconditional loads
                        const float x = part[(int64_t)(s + u * G) * L + l + (k < nk ? k : nk - 1)];
                        v[u][k] = k < nk ? x : 0.f;
                    }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[k] += (double)v[u][k];
            }
            for (; s < S; s += G) {
                const float* p = part + (int64_t)s * L + l;
                float v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float x = p[k < nk ? k : nk - 1];
                    v[k] = k < nk ? x : 0.f;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] += (double)v[k];
            }
        }
    }
    __shared__ double red[4][512];
#pragma unroll
    for (int k = 0; k < 4; ++k) red[k][threadIdx.x] = acc[k];
    __syncthreads();
    for (int half = G / 2; half > 0; half >>= 1) {
        if (g < half) {
#pragma unroll
            for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + half * LQ];
        }
        __syncthreads();
    }
    if (g == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (l + k < L) out[l + k] = (float)red[k][q];
    }
}
}  // namespace

int reduce_slabs_pair(const float* part_a, int64_t la, float* out_a, const float* part_b, int64_t lb, float* out_b,
                      int S, hipStream_t stream) {
    UNET_CHECK_ARG(S >= 1 && la >= 1 && lb >= 1 && part_a && part_b && out_a && out_b, "reduce_slabs_pair: bad args");
    constexpr int LQ = 16;  // output quads per block (512 threads / 32 slab groups)
    SlabArr a{part_a, la, out_a, (int)cdiv(cdiv(la, 4), LQ),
              la % 4 == 0 && (reinterpret_cast<uintptr_t>(part_a) & 15) == 0};
    SlabArr b{part_b, lb, out_b, (int)cdiv(cdiv(lb, 4), LQ),
              lb % 4 == 0 && (reinterpret_cast<uintptr_t>(part_b) & 15) == 0};
    reduce_pair_kernel<<<(unsigned)(a.nblk + b.nblk), 512, 0, stream>>>(a, b, S);
    UNET_CHECK_LAUNCH("reduce_slabs_pair");
    return 0;
}

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_view(const unet_view* v, const char* op, bool need_vec4) {
    UNET_CHECK_ARG(v != nullptr, "%s: null view", op);
    UNET_CHECK_ARG(v->mode >= UNET_VIEW_PLAIN && v->mode <= UNET_VIEW_CONCAT, "%s: bad view mode %d", op, v->mode);
    UNET_CHECK_ARG(v->src0 != nullptr && v->c0 > 0, "%s: view needs src0 and c0 > 0", op);
    if (v->mode == UNET_VIEW_BNRELU || v->mode == UNET_VIEW_POOL_BNRELU)
        UNET_CHECK_ARG(v->scale0 && v->shift0, "%s: BN view needs scale0/shift0", op);
    if (v->mode == UNET_VIEW_CONCAT) {
        UNET_CHECK_ARG(v->src1 && v->scale1 && v->shift1 && v->c1 > 0, "%s: CONCAT view needs src1/scale1/shift1/c1",
                       op);
        UNET_CHECK_ARG(v->c0 % 4 == 0 || (v->c0 % 4 != 0 && !need_vec4), "%s: CONCAT c0 must be a multiple of 4", op);
    }
    UNET_CHECK_ARG(v->drop_rate >= 0.f && v->drop_rate < 1.f, "%s: drop_rate %f out of [0,1)", op, v->drop_rate);
    if (need_vec4) {
        const int C = v->c0 + (v->mode == UNET_VIEW_CONCAT ? v->c1 : 0);
        UNET_CHECK_ARG(C % 4 == 0, "%s: channels (%d) must be a multiple of 4", op, C);
    }
    return 0;
}

int reduce_slabs(float* part, int S, int64_t L, float* out, int64_t row, int64_t ld_out, hipStream_t stream) {
    UNET_CHECK_ARG(S >= 1 && L >= 1 && row >= 1, "reduce_slabs: bad sizes");
    const bool vec = L % 4 == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0;
    int64_t sp = L;  // slab pitch
    if (vec) {
        // groups per output quad: enough threads for ~256K loads in flight, at most 32, at most S
        const int64_t quads = L / 4;
        // long, narrow reductions (< 64 blocks of 16 quads x 32 groups would walk > 256 slabs each):
        // in-place chunk levels of 16 slabs first
        while (S > 256 && quads < 64 * 16) {
            constexpr int CH = 16;
            const dim3 grid((unsigned)cdiv(quads, 256), (unsigned)cdiv(S, CH));
            reduce_chunk_kernel<<<grid, 256, 0, stream>>>(part, S, L, sp, CH);
            UNET_CHECK_LAUNCH("reduce_slabs(chunk)");
            S = (int)cdiv(S, CH);
            sp *= CH;
        }
        int G = 1;
        while (G < 32 && G < S && quads * G < 262144) G *= 2;
        if (G == 1 || S <= 8)
            reduce_cols4_kernel<<<(unsigned)cdiv(L, 1024), 256, 0, stream>>>(part, S, L, sp, out, row, ld_out);
        else if (G == 2 || G == 4)
            reduce_grp4_kernel<4><<<(unsigned)cdiv(quads, 128), 512, 0, stream>>>(part, S, L, sp, out, row, ld_out);
        else if (G == 8)
            reduce_grp4_kernel<8><<<(unsigned)cdiv(quads, 64), 512, 0, stream>>>(part, S, L, sp, out, row, ld_out);
        else if (G == 16)
            reduce_grp4_kernel<16><<<(unsigned)cdiv(quads, 32), 512, 0, stream>>>(part, S, L, sp, out, row, ld_out);
        else
            reduce_grp4_kernel<32><<<(unsigned)cdiv(quads, 16), 512, 0, stream>>>(part, S, L, sp, out, row, ld_out);
    } else if (L == 1) {
        reduce_one_kernel<<<1, 1024, 0, stream>>>(part, S, out, row, ld_out);
    } else {
        reduce_slabs_kernel<<<(unsigned)cdiv(L, 64), 1024, 0, stream>>>(part, S, L, sp, out, row, ld_out);
    }
    UNET_CHECK_LAUNCH("reduce_slabs");
    return 0;
}

}  // namespace unet

#ifdef UNET_LAB_BUILD
#include <cstdlib>
namespace unet {
int lab_knob(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
}  // namespace unet
#endif

namespace unet {
namespace {
__global__ __launch_bounds__(256) void copy_strided_kernel(const float* __restrict__ src, int64_t rows, int cols,
                                                           int64_t src_ld, float* __restrict__ dst, int64_t dst_ld) {
    const int64_t n = rows * cols;
    if (n < (int64_t(1) << 31)) {  // 32-bit index math (a 64-bit division per element doubled the launch)
        const unsigned uc = (unsigned)cols;
        for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < (unsigned)n; i += gridDim.x * 256u) {
            const unsigned r = i / uc, c = i - r * uc;
            dst[(int64_t)r * dst_ld + c] = src[(int64_t)r * src_ld + c];
        }
        return;
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols, c = i - r * cols;
        dst[r * dst_ld + c] = src[r * src_ld + c];
    }
}
// rows of <= 4 floats into 16-B aligned rows of 4 (the image's channel padding): one float4 store
// per row, the columns past `cols` kept as they are
__global__ __launch_bounds__(256) void copy_rows4_kernel(const float* __restrict__ src, int64_t rows, int cols,
                                                         int64_t src_ld, float4* __restrict__ dst) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < rows; r += (int64_t)gridDim.x * 256) {
        float4 v = dst[r];
        const float* p = src + r * src_ld;
        v.x = p[0];
        if (cols > 1) v.y = p[1];
        if (cols > 2) v.z = p[2];
        if (cols > 3) v.w = p[3];
        dst[r] = v;
    }
}
}  // namespace
}  // namespace unet

extern "C" int unet_copy_strided(const float* src, int64_t rows, int cols, int64_t src_ld, float* dst, int64_t dst_ld,
                                 unet_stream_t stream) {
    UNET_CHECK_ARG(src && dst, "unet_copy_strided: null pointer");
    UNET_CHECK_ARG(rows >= 0 && cols >= 0 && src_ld >= cols && dst_ld >= cols, "unet_copy_strided: bad sizes");
    const int64_t n = rows * cols;
    if (n == 0) return 0;
    if (cols <= 4 && dst_ld == 4 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const int64_t blocks = (rows + 255) / 256 < 4096 ? (rows + 255) / 256 : 4096;
        unet::copy_rows4_kernel<<<(unsigned)blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(
            src, rows, cols, src_ld, reinterpret_cast<float4*>(dst));
        UNET_CHECK_LAUNCH("unet_copy_strided");
        return 0;
    }
    const int64_t blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    unet::copy_strided_kernel<<<(unsigned)blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(src, rows, cols, src_ld,
                                                                                              dst, dst_ld);
    UNET_CHECK_LAUNCH("unet_copy_strided");
    return 0;
}

namespace unet {
namespace {
struct SplitTable {
    int n;
    int64_t src[UNET_SPLIT_MAX_SEGS], dst[UNET_SPLIT_MAX_SEGS];
    int rows[UNET_SPLIT_MAX_SEGS], cols[UNET_SPLIT_MAX_SEGS];
    unsigned char keep[UNET_SPLIT_MAX_SEGS];  // per segment: planes in the source layout (else transposed)
};
// dst planes [3][cols][rows] (bf16 bits) of src [rows][cols]: a 32 x 32 tile per block through LDS,
// read along cols and written along rows (blockIdx.y = segment)
// (KEEP: planes [3][rows][cols] in the source layout, for the operands a GEMM stages k-contiguous as
// they are: the dgrad reads pw_kernel[ci][co] with k = co)
__global__ __launch_bounds__(256) void split_x3_kernel(const float* __restrict__ src, SplitTable t,
                                                       unsigned short* __restrict__ dst) {
    __shared__ float T[32][33];
    const int s = blockIdx.y;
    const bool KEEP = t.keep[s] != 0;  // (uniform per block)
    const int rows = t.rows[s], cols = t.cols[s];
    const int tr = (rows + 31) / 32, tc = (cols + 31) / 32;
    const float* S = src + t.src[s];
    unsigned short* D = dst + t.dst[s];
    const int64_t plane = (int64_t)rows * cols;
    for (int tile = blockIdx.x; tile < tr * tc; tile += gridDim.x) {
        const int r0 = (tile / tc) * 32, c0 = (tile % tc) * 32;
        __syncthreads();
        for (int i = threadIdx.x; i < 1024; i += 256) {
            const int r = r0 + (i >> 5), c = c0 + (i & 31);
            T[i >> 5][i & 31] = (r < rows && c < cols) ? S[(int64_t)r * cols + c] : 0.f;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 1024; i += 256) {
            // transposed planes: consecutive threads walk r (the destination's contiguous axis);
            // KEEP: they walk c, as the source
            const int c = c0 + (KEEP ? (i & 31) : (i >> 5)), r = r0 + (KEEP ? (i >> 5) : (i & 31));
            if (r < rows && c < cols) {
                const float x = T[r - r0][c - c0];
                const unsigned h = bf16_bits(x);
                const float rr = x - bf16_val(h);
                const unsigned m = bf16_bits(rr);
                const unsigned l = bf16_bits(rr - bf16_val(m));
                const int64_t o = KEEP ? (int64_t)r * cols + c : (int64_t)c * rows + r;
                D[o] = (unsigned short)h;
                D[plane + o] = (unsigned short)m;
                D[2 * plane + o] = (unsigned short)l;
            }
        }
    }
}
}  // namespace
}  // namespace unet

namespace {
// keep: 0 every segment transposed, 1 every segment kept, -1 per segment (segs of 5: ..., keep flag)
int split_x3(const float* src, const int64_t* segs, int nseg, unsigned short* dst, unet_stream_t stream, int keep) {
    const int F = keep < 0 ? 5 : 4;
    UNET_CHECK_ARG(src && segs && dst && nseg > 0 && nseg <= UNET_SPLIT_MAX_SEGS, "unet_split_x3: bad arguments");
    unet::SplitTable t{};
    t.n = nseg;
    int maxtiles = 1;
    for (int i = 0; i < nseg; ++i) {
        const int64_t so = segs[F * i], rows = segs[F * i + 1], cols = segs[F * i + 2], doff = segs[F * i + 3];
        UNET_CHECK_ARG(so >= 0 && doff >= 0 && rows > 0 && cols > 0 && rows < (1 << 30) && cols < (1 << 30),
                       "unet_split_x3: bad segment %d", i);
        UNET_CHECK_ARG(doff % 8 == 0, "unet_split_x3: segment %d destination must be 16-B aligned", i);
        t.src[i] = so;
        t.dst[i] = doff;
        t.rows[i] = (int)rows;
        t.cols[i] = (int)cols;
        t.keep[i] = (unsigned char)(keep < 0 ? segs[F * i + 4] != 0 : keep);
        const int64_t tiles = ((rows + 31) / 32) * ((cols + 31) / 32);
        if (tiles > maxtiles) maxtiles = tiles > 1024 ? 1024 : (int)tiles;
    }
    const dim3 grid((unsigned)maxtiles, (unsigned)nseg);
    unet::split_x3_kernel<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(src, t, dst);
    UNET_CHECK_LAUNCH("unet_split_x3");
    return 0;
}
}  // namespace

extern "C" int unet_split_x3(const float* src, const int64_t* segs, int nseg, unsigned short* dst,
                             unet_stream_t stream) {
    return split_x3(src, segs, nseg, dst, stream, 0);
}
extern "C" int unet_split_x3_keep(const float* src, const int64_t* segs, int nseg, unsigned short* dst,
                                  unet_stream_t stream) {
    return split_x3(src, segs, nseg, dst, stream, 1);
}
extern "C" int unet_split_x3_mixed(const float* src, const int64_t* segs, int nseg, unsigned short* dst,
                                   unet_stream_t stream) {
    return split_x3(src, segs, nseg, dst, stream, -1);
}

extern "C" int unet_abi_version(void) { return UNET_ABI_VERSION; }
extern "C" const char* unet_last_error(void) { return unet::g_err; }

// Cross-stream ordering events for the two-stream backward.  Both streams live on one device, so
// the device-scope release of a marker is enough: no timing, no system-scope fence (the default
// event's system-scope writeback/invalidate stalls the recording stream for several us).
extern "C" int unet_event_create(void** event) {
    UNET_CHECK_ARG(event, "unet_event_create: null out pointer");
    hipEvent_t e = nullptr;
    hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
    if (rc != hipSuccess) {
        unet::set_error("unet_event_create: %s", hipGetErrorString(rc));
        return (int)rc;
    }
    *event = e;
    return 0;
}
extern "C" int unet_event_destroy(void* event) {
    if (!event) return 0;
    return (int)hipEventDestroy(static_cast<hipEvent_t>(event));
}
extern "C" int unet_stream_wait_stream(unet_stream_t waiter, unet_stream_t producer, void* event) {
    UNET_CHECK_ARG(event, "unet_stream_wait_stream: null event");
    hipEvent_t e = static_cast<hipEvent_t>(event);
    hipError_t rc = hipEventRecord(e, static_cast<hipStream_t>(producer));
    if (rc == hipSuccess) rc = hipStreamWaitEvent(static_cast<hipStream_t>(waiter), e, 0);
    if (rc != hipSuccess) {
        unet::set_error("unet_stream_wait_stream: %s", hipGetErrorString(rc));
        return (int)rc;
    }
    return 0;
}
