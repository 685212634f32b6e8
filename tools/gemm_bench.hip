// gemm_bench.hip -- microbenchmark of the tiled MFMA GEMM (csrc/gemm.hip,
// included directly) on the encoder / prefill shapes: TFLOP/s per tile config.
#include "../qwen3-asr.cpp_amd/csrc/gemm.hip"

#include <cstdio>
#include <cstdlib>

namespace qasr { bool launch_gemv1(int, const GemvArgs &, hipStream_t) { return false; } }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace qasr;

template <int BM, int BN, int KS, int EPI>
static void run(const char *tag, GemmArgs g, hipStream_t s) {
    if (g.N % BN || g.K % (32 * KS)) { printf("  %-6s %3dx%-3d KS%d  n/a\n", tag, BM, BN, KS); return; }
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    const int NREP = 20;
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((gemm_kernel<BM, BN, KS, AM_DENSE, EPI>), grid, dim3(256), 0, s, g);
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int it = 0; it < 3; it++) {
        CK(hipEventRecord(a, s));
        for (int r = 0; r < NREP; r++) hipLaunchKernelGGL((gemm_kernel<BM, BN, KS, AM_DENSE, EPI>), grid, dim3(256), 0, s, g);
        CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    const double us = best * 1e3 / NREP, fl = 2.0 * g.M * g.N * g.K;
    printf("  %-6s %3dx%-3d KS%d  %8.1f us  %7.1f TFLOP/s  grid %dx%d\n", tag, BM, BN, KS, us, fl / us * 1e-6, grid.x, grid.y);
}

int main() {
    hipStream_t s; CK(hipStreamCreate(&s));
    struct Sh { const char *name; int M, N, K; };
    Sh shapes[] = {{"prefill qkv b1", 1211, 4096, 1024}, {"prefill o b1", 1211, 1024, 2048}, {"prefill dn b1", 1211, 1024, 3072},
                   {"enc qkv b1", 1196, 2688, 896}, {"enc fc1 b1", 1196, 3584, 896}, {"enc fc2 b1", 1196, 896, 3584},
                   {"prefill qkv b64", 25920, 4096, 1024}, {"prefill dn b64", 25920, 1024, 3072}, {"enc fc1 b64", 24960, 3584, 896}};
    uint16_t *A, *W; float *out; uint16_t *o16;
    CK(hipMalloc(&A, (size_t)25920 * 4096 * 2)); CK(hipMalloc(&W, (size_t)6144 * 4096 * 2));
    CK(hipMalloc(&out, (size_t)25920 * 6144 * 4)); CK(hipMalloc(&o16, (size_t)25920 * 6144 * 2));
    CK(hipMemset(A, 0x11, (size_t)25920 * 4096 * 2)); CK(hipMemset(W, 0x22, (size_t)6144 * 4096 * 2));
    for (const Sh &sh : shapes) {
        GemmArgs g{};
        g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.M = sh.M; g.N = sh.N; g.K = sh.K; g.out_f32 = out; g.ldo = sh.N;
        printf("%s  M=%d N=%d K=%d\n", sh.name, sh.M, sh.N, sh.K);
        run<64, 64, 2, EPI_F32>("f32", g, s);
        run<64, 64, 4, EPI_F32>("f32", g, s);
        run<128, 64, 2, EPI_F32>("f32", g, s);
        run<64, 128, 2, EPI_F32>("f32", g, s);
        run<128, 128, 2, EPI_F32>("f32", g, s);
        run<128, 128, 1, EPI_F32>("f32", g, s);
        run<96, 64, 2, EPI_F32>("f32", g, s);
        run<64, 96, 2, EPI_F32>("f32", g, s);
        run<128, 96, 2, EPI_F32>("f32", g, s);
    }
    return 0;
}
