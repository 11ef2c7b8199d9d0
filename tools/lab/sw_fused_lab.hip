// Knock-out timing of the fused 64-output block backward (csrc/sepwgrad.hip, unet_sepconv_bwd_fused)
// at enc1_block2's shape (16 x 256 x 256, BN+ReLU view of 64 channels) and dec1_block1's (concat
// view 64 + 64).  Build one binary per SW_KO value (sepwgrad.hip's knock-out bits).  Lab only.
#include "sepwgrad.hip"
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
static float* dalloc(size_t n) { float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemset(d, 0, n * 4)); return d; }
static void shape(int cat) {
    const int n = 16, h = 256, w = 256, C = cat ? 128 : 64, CO = 64;
    const size_t M = (size_t)n * h * w;
    unet_view v{};
    v.mode = cat ? UNET_VIEW_CONCAT : UNET_VIEW_BNRELU;
    v.c0 = cat ? 64 : C;
    v.src0 = dalloc(M * v.c0); v.scale0 = dalloc(v.c0); v.shift0 = dalloc(v.c0);
    if (cat) { v.c1 = 64; v.src1 = dalloc(M * 64); v.scale1 = dalloc(64); v.shift1 = dalloc(64); }
    float *dk = dalloc(9 * C), *pk = dalloc((size_t)C * CO), *da = dalloc(M * CO), *z = dalloc(M * CO);
    float *sc = dalloc(CO), *sh = dalloc(CO), *coef = dalloc(3 * CO), *dy = dalloc(M * C);
    float *ddk = dalloc(9 * C), *dpk = dalloc((size_t)C * CO);
    const size_t wsb = unet_sepconv_bwd_filter_workspace(n, h, w, C, CO);
    float* ws = dalloc(wsb / 4 + 64);
    auto run = [&] {
        if (unet_sepconv_bwd_fused(&v, n, h, w, dk, pk, da, z, sc, sh, coef, CO, dy, ddk, dpk, ws, wsb, 0)) {
            printf("err %s\n", unet_last_error());
            exit(1);
        }
    };
    for (int i = 0; i < 3; ++i) run();
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < 20; ++i) run();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"shape\": \"%s\", \"ko\": %d, \"us\": %.1f}\n", cat ? "dec1_block1 128->64" : "enc1_block2 64->64", SW_KO,
           ms * 1e3 / 20);
}
int main() {
    shape(0);
    shape(1);
    return 0;
}
