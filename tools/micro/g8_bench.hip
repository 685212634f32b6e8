// g8_bench.hip -- the 256 x 256 8-phase GEMM (csrc/gemm8p.h) on the encoder /
// prefill shapes: us per launch and TFLOP/s per epilogue and with no stores at
// all; EPI_F32 (+ bias + residual) checked against a naive fp32-accumulating
// reference within a tolerance (bit identity with the other GEMM tiles: the
// engine's option tests, tests/test_gpu_full.py).
#include "../../qwen3-asr.cpp_amd/csrc/gemm8p.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace qasr;

__global__ void naive_ref(const uint16_t *A, const uint16_t *W, int M, int N, int K, float *out) {
    const int n = blockIdx.x * 64 + threadIdx.x, m = blockIdx.y;
    if (n >= N) return;
    float acc = 0.f;
    for (int k = 0; k < K; k++) acc += (float)__builtin_bit_cast(_Float16, A[(long)m * K + k]) * (float)__builtin_bit_cast(_Float16, W[(long)n * K + k]);
    out[(long)m * N + n] = acc;
}

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

template <int EPI>
static void timed(GemmArgs g, hipStream_t s, const char *name) {
    // host check before any launch: the output this EPI writes exists
    const bool f32_out = EPI == EPI_F32 || EPI == EPI_SWIGLU_F32;
    if ((f32_out && !g.out_f32) || (!f32_out && !g.out_f16) || (EPI == EPI_GELU_F16 && !g.gelu) || (g.res && g.ldr < g.N)) {
        printf("  %-10s bad arguments\n", name);
        exit(1);
    }
    const double us = timeit([&] { run_gemm8p<EPI>(g, s); }, s), fl = 2.0 * g.M * g.N * g.K;
    printf("  %-10s %7.1f us %6.1f TF\n", name, us, fl / us * 1e-6);
}

int main(int argc, char **argv) {
    hipStream_t s; CK(hipStreamCreate(&s));
    struct Sh { const char *name; int M, N, K; };
    Sh shapes[] = {{"enc qkv b64", 24960, 2688, 896},    {"enc fc1 b64", 24960, 3584, 896},     {"enc fc2 b64", 24960, 896, 3584},
                   {"enc o b64", 24960, 896, 896},       {"prefill qkv b64", 25920, 4096, 1024}, {"prefill dn b64", 25920, 1024, 3072},
                   {"prefill o b64", 25920, 1024, 2048}, {"prefill gu b64", 25920, 6144, 1024},  {"odd M", 2500, 1024, 1024},
                   {"4096^3", 4096, 4096, 4096}};
    const size_t MA = (size_t)25920 * 4096, MW = (size_t)6144 * 4096, MO = (size_t)25920 * 6144;
    for (const Sh &sh : shapes)
        if ((size_t)sh.M * sh.K > MA || (size_t)sh.N * sh.K > MW || (size_t)sh.M * sh.N > MO) { printf("buffer too small for %s\n", sh.name); return 1; }
    uint16_t *A, *W, *lut; float *o1, *o2, *ref, *bias, *res;
    CK(hipMalloc(&A, MA * 2)); CK(hipMalloc(&W, MW * 2)); CK(hipMalloc(&o1, MO * 4)); CK(hipMalloc(&o2, MO * 4));
    CK(hipMalloc(&ref, MO * 4)); CK(hipMalloc(&bias, 8192 * 4)); CK(hipMalloc(&res, MO * 4)); CK(hipMalloc(&lut, 65536 * 2));
    {
        std::vector<_Float16> h(MW);
        unsigned x = 12345u;
        for (size_t i = 0; i < MW; i++) { x = x * 1664525u + 1013904223u; h[i] = (_Float16)(((x >> 9) * (1.0f / 8388608.0f)) * 2.0f - 1.0f); }
        CK(hipMemcpy(A, h.data(), MA * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(W, h.data() + 7, (MW - 7) * 2, hipMemcpyHostToDevice));
        std::vector<float> b(8192);
        for (int i = 0; i < 8192; i++) b[i] = 0.01f * (i % 97) - 0.4f;
        CK(hipMemcpy(bias, b.data(), b.size() * 4, hipMemcpyHostToDevice));
        std::vector<uint16_t> l(65536);
        for (int i = 0; i < 65536; i++) l[i] = (uint16_t)(i * 40503u >> 3);
        CK(hipMemcpy(lut, l.data(), l.size() * 2, hipMemcpyHostToDevice));
        std::vector<float> r((size_t)4096 * 8192);
        for (size_t i = 0; i < r.size(); i++) r[i] = 0.001f * (float)(i % 1999) - 1.0f;
        CK(hipMemcpy(res, r.data(), r.size() * 4, hipMemcpyHostToDevice));
    }
    for (const Sh &sh : shapes) {
        GemmArgs g{};
        g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.M = sh.M; g.N = sh.N; g.K = sh.K; g.ldo = sh.N; g.ldo16 = sh.N;
        g.out_f32 = o1;
        g.out_f16 = (uint16_t *)o2;
        printf("%s  M=%d N=%d K=%d\n", sh.name, sh.M, sh.N, sh.K);
        const double fl = 2.0 * sh.M * sh.N * sh.K;
        double us = timeit([&] { run_gemm8p<G8_EPI_NONE>(g, s); }, s);
        printf("  no stores  %7.1f us %6.1f TF\n", us, fl / us * 1e-6);
        // accuracy of EPI_F32 + bias + residual against the naive reference (first 512 rows)
        {
            const int Mr = sh.M < 512 ? sh.M : 512;
            hipLaunchKernelGGL(naive_ref, dim3((sh.N + 63) / 64, Mr), dim3(64), 0, s, A, W, Mr, sh.N, sh.K, ref);
            GemmArgs gb = g; gb.bias = bias; gb.res = res; gb.ldr = sh.N;
            run_gemm8p<EPI_F32>(gb, s);
            CK(hipStreamSynchronize(s));
            std::vector<float> x((size_t)Mr * sh.N), y((size_t)Mr * sh.N), r((size_t)Mr * sh.N), b(sh.N);
            CK(hipMemcpy(x.data(), o1, x.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(y.data(), ref, y.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(r.data(), res, r.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), bias, b.size() * 4, hipMemcpyDeviceToHost));
            double m = 0;
            for (size_t i = 0; i < x.size(); i++) {
                const double e = fabs((double)x[i] - ((double)y[i] + b[i % sh.N] + r[i]));
                if (!(e <= m)) m = e;
            }
            printf("  f32+bias+res vs naive fp32 reference (first %d rows): max |diff| %.3g %s\n", Mr, m, m < 1e-2 ? "ok" : "BAD");
        }
        timed<EPI_F32>(g, s, "f32");
        GemmArgs gb = g; gb.bias = bias; gb.res = res; gb.ldr = sh.N;
        timed<EPI_F32>(gb, s, "f32+b+res");
        GemmArgs gr = g; gr.res = res; gr.ldr = sh.N;
        timed<EPI_F32>(gr, s, "f32+res");
        GemmArgs gg = g; gg.bias = bias; gg.gelu = lut;
        timed<EPI_GELU_F16>(gg, s, "gelu f16");
        timed<EPI_F16>(g, s, "f16");
        GemmArgs gs = g; gs.ldo = sh.N / 2; gs.ldo16 = sh.N / 2;
        timed<EPI_SWIGLU_F16>(gs, s, "swiglu f16");
    }
    return 0;
}
