// Shared definitions of the fused SeparableConv2D forward kernels (sepconv.hip: the LDS-A-tile
// schedule; sepconv_rk.hip: the register-A schedule).  Reference model/u_net.py:14-23.
#pragma once
#include "view.h"

namespace unet {
namespace sep {

constexpr int TH = 8, TW = 16;            // pixel rectangle of one M tile
constexpr int HHp = TH + 2, HWp = TW + 2; // halo
constexpr int BK = 16;                    // channels per k-stage
enum { E_STORE = 0, E_STATS = 1 };

__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

struct SepArgs {
    DView x;
    int N, H, W, Cin, Cout;
    const float* dk;  // (3,3,Cin,1)
    const float* pk;  // (1,1,Cin,Cout): B(k, n) = pk[k*Cout + n] (n-contiguous)
    float* y;         // optional (N,H,W,Cin)
    float* z;         // (N,H,W,Cout)
    float2* stats;    // [M/128][Cout]
    const unsigned short* pkx;  // optional bf16x3 split of pk: planes [3][Cout][Cin] (unet_split_x3)
    float* zsel;         // optional (N,H/2,W/2,Cout): the 2x2 pooling selection of z (pool_select_kernel)
    const float* gamma;  // zsel: BN gamma (its sign orders the window), NULL = no BN (max)
};

// The raw z value of a 2x2 window that the max-pool of relu(z * s + b) takes, with s of the sign of
// gamma: the max where gamma >= 0 (+0 included), the min where gamma < 0.  fmaf is monotone in z,
// so relu(fmaf(sel, s, b)) is bitwise the max over the window of relu(fmaf(z, s, b)).
__device__ __forceinline__ float pool_sel(float a, float b, float c, float d, bool neg) {
    return neg ? fminf(fminf(a, b), fminf(c, d)) : fmaxf(fmaxf(a, b), fmaxf(c, d));
}

// register-A schedule (sepconv_rk.hip): returns 0, or -1 if the mode/shape has no such kernel.
// With a.pkx (and Cin % 16 == 0, no max-pool view) the split-precision (bf16x6) variant runs.
int launch_rk(const SepArgs& a, int mode, bool drop, bool stats, bool write_y, hipStream_t st);
bool rk_x6_supported(int mode, int cin);
bool rk_supported(int mode, int cin, int cout);
// persistent split-precision schedule (sepconv_px.hip) for 64 / 128 input and output channels:
// returns 0, or -1 if the shape has no such kernel (needs a.pkx)
bool px_supported(const SepArgs& a, int mode, bool all_shapes);
int launch_px(const SepArgs& a, int mode, bool drop, bool stats, bool write_y, hipStream_t st);

}  // namespace sep
}  // namespace unet
