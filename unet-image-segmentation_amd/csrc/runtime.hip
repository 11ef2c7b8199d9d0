// Error reporting, view validation and the deterministic slab reduction shared by
// every op of libunet_hip.so.
#include <stdarg.h>

#include "view.h"

namespace unet {

namespace {
thread_local char g_err[512] = "";

// out[l] = sum_s part[s][l], s in a fixed order.  Block = 64 columns x G s-groups;
// each thread sums s = g, g+G, ... in double, then group 0 adds the G partials in order.
__global__ __launch_bounds__(1024) void reduce_slabs_kernel(const float* __restrict__ part, int S, int64_t L,
                                                            float* __restrict__ out, int64_t row, int64_t ld_out) {
    const int G = blockDim.x / 64;
    const int lane = threadIdx.x & 63;
    const int g = threadIdx.x >> 6;
    const int64_t l = (int64_t)blockIdx.x * 64 + lane;
    double acc = 0.0;
    if (l < L) {
        int s = g;
        for (; s + 3 * G < S; s += 4 * G) {
            float a0 = part[(int64_t)s * L + l];
            float a1 = part[(int64_t)(s + G) * L + l];
            float a2 = part[(int64_t)(s + 2 * G) * L + l];
            float a3 = part[(int64_t)(s + 3 * G) * L + l];
            acc += (double)a0;
            acc += (double)a1;
            acc += (double)a2;
            acc += (double)a3;
        }
        for (; s < S; s += G) acc += (double)part[(int64_t)s * L + l];
    }
    __shared__ double red[16][64];
    red[g][lane] = acc;
    __syncthreads();
    if (g == 0 && l < L) {
        double t = red[0][lane];
        for (int k = 1; k < G; ++k) t += red[k][lane];
        out[(l / row) * ld_out + (l % row)] = (float)t;
    }
}
}  // namespace

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

int reduce_slabs(const float* part, int S, int64_t L, float* out, int64_t row, int64_t ld_out, hipStream_t stream) {
    UNET_CHECK_ARG(S >= 1 && L >= 1 && row >= 1, "reduce_slabs: bad sizes");
    int G = S < 16 ? S : 16;
    dim3 grid((unsigned)cdiv(L, 64));
    reduce_slabs_kernel<<<grid, 64 * G, 0, stream>>>(part, S, L, out, row, ld_out);
    UNET_CHECK_LAUNCH("reduce_slabs");
    return 0;
}

}  // namespace unet

extern "C" int unet_abi_version(void) { return UNET_ABI_VERSION; }
extern "C" const char* unet_last_error(void) { return unet::g_err; }
