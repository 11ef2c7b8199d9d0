// Timing lab for the rows GEMM (pointwise fwd / BN-backward dgrad shapes of the U-Net at
// batch 16, 256x256).  Includes the product gemm.hip so its kernels can be instantiated with
// other tile parameters; candidate kernels are added below.  Prints us and TF/s per variant,
// and max |diff| against the product kernel's output.
#include "gemm.hip"
#include <vector>
#include <algorithm>
#include <cmath>
#include <cstdlib>

using namespace unet;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static float* dalloc(size_t n, float scale, unsigned seed) {
    std::vector<float> h(n);
    srand(seed);
    for (size_t i = 0; i < n; ++i) h[i] = scale * ((float)rand() / RAND_MAX * 2.f - 1.f);
    float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}
static double maxdiff(const float* a, const float* b, size_t n) {
    std::vector<float> x(n), y(n);
    CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
    double m = 0, r = 0;
    for (size_t i = 0; i < n; ++i) { m = fmax(m, fabs((double)x[i] - y[i])); r = fmax(r, fabs((double)y[i])); }
    return m / (r + 1e-30);
}

template <class F> static double timeit(F f, int it = 20) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a)); for (int i = 0; i < it; ++i) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms * 1e3 / it;
}

#include "gemm_v2.inc"
#include "gemm_wv2.inc"
#include "gemm_lab_variants.inc"

template <int BP, int BQ, int BK, bool V2>
static void wlaunch(const WgradArgs& a, const WgradPlan& w) {
    dim3 grid((unsigned)w.tiles, (unsigned)w.S);
    if (V2) gemm_wgrad_v2<BP, BQ, BK, W_PLAIN, false, W_PLAIN, false><<<grid, 256>>>(a);
    else gemm_wgrad_vec<BP, BQ, W_PLAIN, false, W_PLAIN, false><<<grid, 256>>>(a);
}
template <int BP, int BQ>
static void wgrad_variants(WgradArgs a, const WgradPlan& w, float* s0, float* s1, double fl, size_t n) {
    a.slab = s0; wlaunch<BP, BQ, 16, false>(a, w); CK(hipDeviceSynchronize());
    auto V = [&](const char* name, auto fn) {
        CK(hipMemset(s1, 0, n * 4));
        double us = timeit([&] { fn(); });
        double d = maxdiff(s1, s0, n);
        printf("  %-34s %8.1f us %7.1f TF/s  diff %.2e\n", name, us, fl / us * 1e-6, d);
    };
    a.slab = s1;
    V("product wgrad_vec", [&] { wlaunch<BP, BQ, 16, false>(a, w); });
    V("v2 BK16", [&] { wlaunch<BP, BQ, 16, true>(a, w); });
    V("v2 BK32", [&] { wlaunch<BP, BQ, 32, true>(a, w); });
}
static void run_wgrad_lab() {
    struct WS { int64_t M; int P, Q; };
    std::vector<WS> ws = {{1048576, 64, 64}, {262144, 64, 128}, {262144, 128, 128}, {65536, 128, 256}, {65536, 256, 256},
                          {16384, 256, 512}, {16384, 512, 512}, {4096, 512, 1024}, {4096, 1024, 1024},
                          {16384, 1024, 512}, {65536, 512, 256}, {262144, 256, 128}, {1048576, 128, 64}};
    for (auto& s : ws) {
        float* A = dalloc(s.M * s.P, 1.f, 11);
        float* B = dalloc(s.M * s.Q, 1.f, 12);
        WgradArgs a{};
        unet_view va{}; va.mode = UNET_VIEW_PLAIN; va.c0 = s.P; va.src0 = A;
        unet_view vb{}; vb.mode = UNET_VIEW_PLAIN; vb.c0 = s.Q; vb.src0 = B;
        a.a = make_dview(va); a.b = make_dview(vb); a.P = s.P; a.Q = s.Q; a.M = s.M;
        WgradPlan w = wgrad_plan(s.M, s.P, s.Q);
        a.mslice = w.mslice;
        const size_t n = (size_t)w.S * s.P * s.Q;
        float *s0, *s1; CK(hipMalloc(&s0, n * 4)); CK(hipMalloc(&s1, n * 4));
        const double fl = 2.0 * s.M * s.P * s.Q;
        printf("WGRAD M=%ld P=%d Q=%d tiles %d S %d mslice %ld\n", (long)s.M, s.P, s.Q, w.tiles, w.S, (long)w.mslice);
        if (w.bp == 128 && w.bq == 128) wgrad_variants<128, 128>(a, w, s0, s1, fl, n);
        else if (w.bp == 128) wgrad_variants<128, 64>(a, w, s0, s1, fl, n);
        else if (w.bq == 128) wgrad_variants<64, 128>(a, w, s0, s1, fl, n);
        else wgrad_variants<64, 64>(a, w, s0, s1, fl, n);
        CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(s0)); CK(hipFree(s1));
        fflush(stdout);
    }
}

int main(int argc, char** argv) {
    if (getenv("LAB_WGRAD")) { run_wgrad_lab(); return 0; }
    struct Shape { int64_t M; int K, N; int mode; };  // mode 0: fwd (B [K][N]), 1: dgrad BN-bwd (B [N][K])
    std::vector<Shape> shapes = {
        {1048576, 64, 64, 0}, {262144, 128, 128, 0}, {65536, 256, 256, 0}, {16384, 512, 512, 0}, {4096, 1024, 1024, 0},
        {16384, 1024, 512, 0}, {16384, 4096, 512, 0}, {65536, 2048, 256, 0}, {8192, 4096, 512, 0}, {32768, 4096, 512, 0},
        {1048576, 64, 64, 1}, {1048576, 64, 128, 1}, {262144, 128, 128, 1}, {262144, 128, 256, 1}, {65536, 256, 256, 1},
        {16384, 512, 512, 1}, {16384, 512, 1024, 1}, {4096, 1024, 1024, 1},
        // Conv2DTranspose fwd (mode 2: N = 4 cout) and data gradient (mode 3: K = 4 cout), batch 16
        {262144, 128, 256, 2}, {65536, 256, 512, 2}, {16384, 512, 1024, 2}, {4096, 1024, 2048, 2},
        {262144, 256, 128, 3}, {65536, 512, 256, 3}, {16384, 1024, 512, 3}, {4096, 2048, 1024, 3},
    };
    const char* only = getenv("LAB_SHAPE");
    int si = -1;
    for (auto& s : shapes) {
        ++si;
        if (only && atoi(only) != si) continue;
        const int lab_batch = getenv("LAB_BATCH") ? atoi(getenv("LAB_BATCH")) : 16;  // shapes are batch 16
        const int64_t M = s.M * lab_batch / 16; const int K = s.K, N = s.N;
        if (getenv("LAB_MODE") && atoi(getenv("LAB_MODE")) != s.mode) continue;
        float* A = dalloc(M * K, 1.f, 1);
        float* Z = dalloc(M * K, 1.f, 2);
        float* B = dalloc((size_t)K * N, 0.1f, 3);
        float* C0; CK(hipMalloc(&C0, M * N * 4));
        float* C1; CK(hipMalloc(&C1, M * N * 4));
        float* side; CK(hipMalloc(&side, M * K * 4));
        float2* stats; CK(hipMalloc(&stats, (M / 32 + 1) * N * 8));
        float* sc = dalloc(K > N ? K : N, 1.f, 4); float* sh = dalloc(K, 0.5f, 5); float* coef = dalloc(3 * K, 0.1f, 6);
        RowsArgs a{};
        unet_view v{}; v.mode = UNET_VIEW_PLAIN; v.c0 = K; v.src0 = A;
        a.a = make_dview(v);
        a.M = M; a.K = K; a.N = N; a.B = B; a.ldc = N;
        const int hw = (int)lround(sqrt((double)(M / lab_batch)));  // convT shapes: square levels
        if (s.mode == 0) { a.sbk = N; a.sbn = 1; a.stats = stats; }
        else if (s.mode == 2) { a.sbk = 1; a.sbn = K; a.bias = sc; a.sH = hw; a.sW = hw; a.sf = N / 4; }
        else if (s.mode == 3) {  // A = dU (n, 2h, 2w, K/4) read unshuffled: M x K elements either way
            a.a.c0 = K / 4; a.uH = hw; a.uW = hw; a.uf = K / 4; a.sbk = N; a.sbn = 1; a.ldc = N; }
        else { a.sbk = 1; a.sbn = K; a.a.sc0 = sc; a.a.sh0 = sh; a.a.rate = 0.2f; a.a.inv_keep = 1.25f; a.a.seed = 77;
               a.z = Z; a.coef = coef; a.side = side; }
        const double fl = 2.0 * M * K * N;
        static const char* mname[4] = {"fwd+stats", "dgrad_bnbwd+drop", "convT fwd", "convT dgrad"};
        printf("M=%ld K=%d N=%d %s\n", (long)M, K, N, mname[s.mode]);
        run_variants(s.mode, a, C0, C1, fl, M * N);
        CK(hipFree(A)); CK(hipFree(Z)); CK(hipFree(B)); CK(hipFree(C0)); CK(hipFree(C1)); CK(hipFree(side));
        CK(hipFree(stats)); CK(hipFree(sc)); CK(hipFree(sh)); CK(hipFree(coef));
        fflush(stdout);
    }
    return 0;
}
