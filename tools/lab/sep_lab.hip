// Lab for the fused separable-conv forward: product schedule vs variants, training settings
// (BN-statistics epilogue + y store), batch 16 / 32 U-Net shapes.
#include "sepconv.hip"
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace unet;
template <class F> static double timeit(F f, int it = 20) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a)); for (int i = 0; i < it; ++i) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); CK(hipGetLastError());
    return ms * 1e3 / it;
}
static float* dalloc(size_t n, float scale) {
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = scale * ((float)((i * 2654435761u) % 1000) / 500.f - 1.f);
    float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}
static double maxdiff(const float* a, const float* b, size_t n) {
    std::vector<float> x(n), y(n);
    CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
    double m = 0; for (size_t i = 0; i < n; ++i) m = fmax(m, fabs((double)x[i] - y[i])); return m;
}
template <int MODE, int BN, int WN, int UNUSED>
static void run(const SepArgs& a) {
    const dim3 grid((unsigned)(a.N * (a.H / 8) * (a.W / 16)), (unsigned)cdiv(a.Cout, BN));
    sepconv_fwd_kernel<MODE, false, E_STATS, BN, WN, true><<<grid, 128 * WN>>>(a);
}
template <int MODE, int BN, int WN>
static void shape(int N, int H, int W, int cin, int cout) {
    const int Hs = MODE == UNET_VIEW_POOL_BNRELU ? 2 * H : H, Ws = MODE == UNET_VIEW_POOL_BNRELU ? 2 * W : W;
    const size_t M = (size_t)N * H * W;
    float* x = dalloc((size_t)N * Hs * Ws * cin, 1.f);
    float* sc = dalloc(cin, 1.f); float* sh = dalloc(cin, 0.2f);
    float* dk = dalloc(9 * cin, 0.3f); float* pk = dalloc((size_t)cin * cout, 0.1f);
    float *y, *z0, *z1, *st;
    CK(hipMalloc(&y, M * cin * 4)); CK(hipMalloc(&z0, M * cout * 4)); CK(hipMalloc(&z1, M * cout * 4));
    CK(hipMalloc(&st, (M / 128 + 1) * cout * 8));
    SepArgs a{};
    unet_view v{}; v.mode = MODE; v.c0 = cin; v.src0 = x; v.scale0 = sc; v.shift0 = sh;
    a.x = make_dview(v); a.N = N; a.H = H; a.W = W; a.Cin = cin; a.Cout = cout; a.dk = dk; a.pk = pk; a.y = y;
    a.stats = (float2*)st;
    const double fl = 2.0 * M * cout * cin + 18.0 * M * cin;
    a.z = z0; run<MODE, BN, WN, 0>(a); CK(hipDeviceSynchronize());
    a.z = z1;
    double t0 = timeit([&] { run<MODE, BN, WN, 0>(a); });
    printf("N=%d %dx%d %d->%d mode %d BN %d: %7.1f us %6.1f TF/s\n", N, H, W, cin, cout, MODE, BN, t0, fl / t0 * 1e-6);
    fflush(stdout);
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(z0)); CK(hipFree(z1)); CK(hipFree(st));
}
int main() {
    for (int N : {16, 32}) {
        shape<UNET_VIEW_BNRELU, 64, 2>(N, 256, 256, 64, 64);
        shape<UNET_VIEW_POOL_BNRELU, 128, 2>(N, 128, 128, 64, 128);
        shape<UNET_VIEW_BNRELU, 128, 2>(N, 128, 128, 128, 128);
        shape<UNET_VIEW_POOL_BNRELU, 256, 4>(N, 64, 64, 128, 256);
        shape<UNET_VIEW_BNRELU, 256, 4>(N, 64, 64, 256, 256);
        shape<UNET_VIEW_POOL_BNRELU, 256, 4>(N, 32, 32, 256, 512);
        shape<UNET_VIEW_BNRELU, 256, 4>(N, 32, 32, 512, 512);
    }
}
