// Knock-out timing of the fused weight-gradient kernel (csrc/sepwgrad.hip) at enc1_block2's
// shape (16 x 256 x 256, 64 -> 64, BN+ReLU view).  Build one binary per SW_KO value.
#include "sepwgrad.hip"
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
static float* dalloc(size_t n) { float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemset(d, 0, n * 4)); return d; }
int main() {
    const int n = 16, h = 256, w = 256, C = 64;
    const size_t M = (size_t)n * h * w;
    unet_view v{}; v.mode = UNET_VIEW_BNRELU; v.c0 = C; v.src0 = dalloc(M * C); v.scale0 = dalloc(C); v.shift0 = dalloc(C);
    float *dk = dalloc(9 * C), *dy = dalloc(M * C), *dz = dalloc(M * C), *ddk = dalloc(9 * C), *dpk = dalloc(C * C);
    const size_t wsb = unet_sepconv_bwd_filter_workspace(n, h, w, C, C);
    float* ws = dalloc(wsb / 4 + 64);
    auto run = [&] { if (unet_sepconv_bwd_filter(&v, n, h, w, dk, dy, dz, C, ddk, dpk, ws, wsb, 0)) { printf("err %s\n", unet_last_error()); exit(1); } };
    for (int i = 0; i < 3; ++i) run();
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a)); for (int i = 0; i < 20; ++i) run(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("SW_KO=%d  %.1f us\n", SW_KO, ms * 1e3 / 20);
    return 0;
}
