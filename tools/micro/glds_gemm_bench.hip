// glds_gemm_bench.hip -- the LDS-DMA ring GEMM (gemm_glds_kernel) against the
// register-staged gemm_kernel on the encoder / prefill shapes: TFLOP/s per
// variant on uniform random fp16 operands, and the max |difference| of the
// fp32 outputs (the two kernels multiply the same fragments in the same k
// order, so they must agree exactly).
#include "../../qwen3-asr.cpp_amd/csrc/gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace qasr { bool launch_gemv1(int, const GemvArgs &, hipStream_t) { return false; } }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace qasr;

static float *g_ref = nullptr;

template <typename F>
static double timeit(F launch, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    launch();
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    const int NREP = 10;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(a, s));
        for (int r = 0; r < NREP; r++) launch();
        CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    return best * 1e3 / NREP;
}

static double maxdiff(const float *d, size_t n) {
    std::vector<float> x(n), y(n);
    CK(hipMemcpy(x.data(), d, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), g_ref, n * 4, hipMemcpyDeviceToHost));
    double m = 0;
    for (size_t i = 0; i < n; i++) { double e = fabs((double)x[i] - y[i]); if (!(e <= m)) m = e; }
    return m;
}

template <int BM, int BN, int KS>
static void ref(GemmArgs g, hipStream_t s) {
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    double us = timeit([&] { hipLaunchKernelGGL((gemm_kernel<BM, BN, KS, AM_DENSE, EPI_F32>), grid, dim3(256), 0, s, g); }, s);
    CK(hipMemcpy(g_ref, g.out_f32, (size_t)g.M * g.N * 4, hipMemcpyDeviceToDevice));
    printf("  regs  %3dx%-3d KS%d      %8.1f us  %7.1f TFLOP/s\n", BM, BN, KS, us, 2.0 * g.M * g.N * g.K / us * 1e-6);
}

template <int BM, int BN, int KS, int NB, int WNW = 2>
static void glds(GemmArgs g, hipStream_t s) {
    if (g.N % BN || g.K % (32 * KS)) { printf("  glds  %3dx%-3d KS%d NB%d W%d  n/a\n", BM, BN, KS, NB, 2 * WNW); return; }
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    CK(hipMemset(g.out_f32, 0, (size_t)g.M * g.N * 4));
    double us = timeit([&] { hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, KS, NB, AM_DENSE, EPI_F32, WNW>), grid, dim3(128 * WNW), 0, s, g); }, s);
    printf("  glds  %3dx%-3d KS%d NB%d W%d  %8.1f us  %7.1f TFLOP/s  maxdiff %.3g\n", BM, BN, KS, NB, 2 * WNW, us,
           2.0 * g.M * g.N * g.K / us * 1e-6, maxdiff(g.out_f32, (size_t)g.M * g.N));
}

template <int EPI = EPI_F32>
static void g8(GemmArgs g, hipStream_t s) {
    if (g.K % 128) { printf("  8p    256x256 n/a\n"); return; }
    CK(hipMemset(g.out_f32, 0, (size_t)g.M * g.N * 4));
    double us = timeit([&] { run_gemm8p<EPI>(g, s); }, s);
    printf("  8p    256x256 BK64      %8.1f us  %7.1f TFLOP/s  maxdiff %.3g\n", us, 2.0 * g.M * g.N * g.K / us * 1e-6,
           maxdiff(g.out_f32, (size_t)g.M * g.N));
    us = timeit([&] { run_gemm8p<G8_EPI_NONE>(g, s); }, s);
    printf("  8p    no stores             %8.1f us  %7.1f TFLOP/s\n", us, 2.0 * g.M * g.N * g.K / us * 1e-6);
}

int main(int argc, char **argv) {
    hipStream_t s; CK(hipStreamCreate(&s));
    struct Sh { const char *name; int M, N, K; };
    Sh shapes[] = {{"enc qkv b64", 24960, 2688, 896}, {"enc fc1 b64", 24960, 3584, 896}, {"enc fc2 b64", 24960, 896, 3584},
                   {"enc o b64", 24960, 896, 896},     {"prefill qkv b64", 25920, 4096, 1024}, {"prefill dn b64", 25920, 1024, 3072},
                   {"prefill o b64", 25920, 1024, 2048}, {"prefill gu b64", 25920, 6144, 1024}, {"enc fc1 b1", 1196, 3584, 896},
                   {"odd M", 2500, 1024, 1024}, {"qkv K2048", 25920, 4096, 2048}, {"qkv K4096", 25920, 4096, 4096},
                   {"4096^3", 4096, 4096, 4096}, {"8192x4096x4096", 8192, 4096, 4096}};
    const size_t MA = (size_t)25920 * 4096, MW = (size_t)4096 * 4096, MO = (size_t)25920 * 6144;   // the largest M x N below (prefill gu)
    uint16_t *A, *W; float *out;
    CK(hipMalloc(&A, MA * 2)); CK(hipMalloc(&W, MW * 2)); CK(hipMalloc(&out, MO * 4)); CK(hipMalloc(&g_ref, MO * 4));
    {
        std::vector<_Float16> h(MA);
        unsigned x = 12345u;
        for (size_t i = 0; i < MA; i++) { x = x * 1664525u + 1013904223u; h[i] = (_Float16)(((x >> 9) * (1.0f / 8388608.0f)) * 2.0f - 1.0f); }
        CK(hipMemcpy(A, h.data(), MA * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(W, h.data() + 7, MW * 2, hipMemcpyHostToDevice));
    }
    const bool b1only = argc > 1 && argv[1][0] == '1';
    const bool quick = argc > 1 && argv[1][0] == 'q';   // the 8-phase kernel only (against the reference tile)
    if (b1only) {   // single-clip (configs[1]) shapes: the dispatch's register tiles against 8-wave LDS-DMA tiles
        Sh b1[] = {{"enc qkv b1", 1196, 2688, 896}, {"enc fc1 b1", 1196, 3584, 896}, {"enc fc2 b1", 1196, 896, 3584},
                   {"enc o b1", 1196, 896, 896},    {"pre qkv b1", 1211, 4096, 1024}, {"pre o b1", 1211, 1024, 2048},
                   {"pre gu b1", 1211, 6144, 1024}, {"pre dn b1", 1211, 1024, 3072}};
        for (const Sh &sh : b1) {
            GemmArgs g{};
            g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.M = sh.M; g.N = sh.N; g.K = sh.K; g.out_f32 = out; g.ldo = sh.N;
            printf("%s  M=%d N=%d K=%d\n", sh.name, sh.M, sh.N, sh.K);
            ref<64, 64, 2>(g, s);
            if (sh.K % 128 == 0) ref<64, 64, 4>(g, s);
            if (sh.N % 96 == 0 || true) ref<96, 64, 2>(g, s);
            glds<128, 128, 1, 2>(g, s);
            glds<128, 128, 1, 4, 4>(g, s);
            glds<128, 128, 1, 3, 4>(g, s);
            glds<64, 128, 1, 4, 4>(g, s);
            glds<128, 64, 1, 4, 4>(g, s);
            glds<64, 64, 1, 4, 2>(g, s);
            glds<64, 256, 1, 4, 4>(g, s);
        }
        return 0;
    }
    for (const Sh &sh : shapes) {
        GemmArgs g{};
        g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.M = sh.M; g.N = sh.N; g.K = sh.K; g.out_f32 = out; g.ldo = sh.N;
        printf("%s  M=%d N=%d K=%d\n", sh.name, sh.M, sh.N, sh.K);
        ref<128, 128, 1>(g, s);
        if (!quick) {
            glds<128, 128, 1, 2>(g, s);
            glds<256, 256, 1, 3, 4>(g, s);
        }
        g8(g, s);
    }
    return 0;
}
