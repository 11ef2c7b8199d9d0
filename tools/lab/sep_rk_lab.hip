// Lab: fused separable-conv forward, product schedule (sepconv_fwd_kernel) vs the register-A
// schedule (sepconv_rk_kernel), training settings (BN-statistics epilogue + y store), on the
// encoder shapes at batch 32 and the decoder/level-0 shapes at batch 16.
// Checks z, y and the statistics of the two kernels against each other (max |diff|) and prints
// time and TF/s.  usage: sep_rk_lab [reps]
#include "sepconv.hip"
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace unet;
static int REPS = 20;
template <class F> static double timeit(F f) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int i = 0; i < REPS; ++i) {
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms * 1e3f);
    }
    CK(hipGetLastError());
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}
static float* dalloc(size_t n, float scale, unsigned salt) {
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = scale * ((float)(((i + salt) * 2654435761u) % 1000) / 500.f - 1.f);
    float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}
static double maxdiff(const float* a, const float* b, size_t n, double* ref = nullptr) {
    std::vector<float> x(n), y(n);
    CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
    double m = 0, r = 0;
    for (size_t i = 0; i < n; ++i) { m = fmax(m, fabs((double)x[i] - y[i])); r = fmax(r, fabs((double)y[i])); }
    if (ref) *ref = r;
    return m;
}
template <int MODE, int BN, int WN>
static void shape(const char* name, int N, int H, int W, int cin, int cout) {
    const int Hs = MODE == UNET_VIEW_POOL_BNRELU ? 2 * H : H, Ws = MODE == UNET_VIEW_POOL_BNRELU ? 2 * W : W;
    const size_t M = (size_t)N * H * W;
    float* x = dalloc((size_t)N * Hs * Ws * cin, 1.f, 1);
    float* sc = dalloc(cin, 1.f, 2); float* sh = dalloc(cin, 0.2f, 3);
    float* dk = dalloc(9 * cin, 0.3f, 4); float* pk = dalloc((size_t)cin * cout, 0.1f, 5);
    float *y0, *y1, *z0, *z1, *s0, *s1;
    const size_t ns = (M / 128 + 1) * cout * 2;
    CK(hipMalloc(&y0, M * cin * 4)); CK(hipMalloc(&y1, M * cin * 4));
    CK(hipMalloc(&z0, M * cout * 4)); CK(hipMalloc(&z1, M * cout * 4));
    CK(hipMalloc(&s0, ns * 4)); CK(hipMalloc(&s1, ns * 4));
    SepArgs a{};
    unet_view v{}; v.mode = MODE; v.c0 = cin; v.src0 = x; v.scale0 = sc; v.shift0 = sh;
    a.x = make_dview(v); a.N = N; a.H = H; a.W = W; a.Cin = cin; a.Cout = cout; a.dk = dk; a.pk = pk;
    const double fl = 2.0 * M * cout * cin + 18.0 * M * cin;
    const double by = 4.0 * ((double)N * Hs * Ws * cin + M * cin + M * cout);
    const double troof = fmax(fl / 157.3e12, by / 8.0e12) * 1e6;
    a.y = y0; a.z = z0; a.stats = (float2*)s0;
    auto old = [&] { launch_tile<MODE, false, BN, WN>(a, true, true, 0); };
    old(); CK(hipDeviceSynchronize());
    const double t0 = timeit(old);
    SepArgs b = a; b.y = y1; b.z = z1; b.stats = (float2*)s1;
    auto rk = [&] { sep::launch_rk(b, MODE, false, true, true, 0); };
    double t2 = 0;
    rk(); CK(hipDeviceSynchronize());
    const double t1 = timeit(rk);
    double rz, ry, rs;
    const double dz = maxdiff(z1, z0, M * cout, &rz), dy = maxdiff(y1, y0, M * cin, &ry),
                 ds = maxdiff(s1, s0, (M / 128) * cout * 2, &rs);
    printf("%-12s N=%d %3dx%-3d %4d->%-4d old %7.1f us (%.3f)  rk %7.1f us (%.3f, %5.1f TF/s)  t_roof %6.1f  "
           "dz %.1e/%.1e dy %.1e ds %.1e  [%.0f]\n", name, N, H, W, cin, cout, t0, troof / t0, t1, troof / t1,
           fl / t1 * 1e-6, troof, dz, rz, dy, ds, t2);
    fflush(stdout);
    CK(hipFree(x)); CK(hipFree(sc)); CK(hipFree(sh)); CK(hipFree(dk)); CK(hipFree(pk));
    CK(hipFree(y0)); CK(hipFree(y1)); CK(hipFree(z0)); CK(hipFree(z1)); CK(hipFree(s0)); CK(hipFree(s1));
}
int main(int argc, char** argv) {
    if (argc > 1) REPS = atoi(argv[1]);
    const int N = 32;
    if (argc > 2) {  // one shape only (PMC passes): enc3_block2
        shape<UNET_VIEW_BNRELU, 256, 4>("enc3_block2", N, 64, 64, 256, 256);
        return 0;
    }
    shape<UNET_VIEW_BNRELU, 64, 2>("enc1_block2", N, 256, 256, 64, 64);

    shape<UNET_VIEW_POOL_BNRELU, 128, 2>("enc2_block1", N, 128, 128, 64, 128);
    shape<UNET_VIEW_BNRELU, 128, 2>("enc2_block2", N, 128, 128, 128, 128);
    shape<UNET_VIEW_POOL_BNRELU, 256, 4>("enc3_block1", N, 64, 64, 128, 256);

    shape<UNET_VIEW_BNRELU, 256, 4>("enc3_block2", N, 64, 64, 256, 256);

    shape<UNET_VIEW_POOL_BNRELU, 256, 4>("enc4_block1", N, 32, 32, 256, 512);
    shape<UNET_VIEW_BNRELU, 256, 4>("enc4_block2", N, 32, 32, 512, 512);
    shape<UNET_VIEW_BNRELU, 256, 4>("dec3_block2", 16, 64, 64, 256, 256);
    shape<UNET_VIEW_BNRELU, 128, 2>("dec2_block2", 16, 128, 128, 128, 128);
    shape<UNET_VIEW_BNRELU, 64, 2>("dec1_block2", 16, 256, 256, 64, 64);
    return 0;
}
