// skinny_bench.hip -- microbenchmark of the decode-batch GEMM tilings
// (csrc/gemm_skinny.hip, included directly so every template is reachable).
// Per shape: hipGraph of NREP dependent launches over NL weight copies
// (> 256 MiB Infinity Cache, so weights stream from HBM as in a decode step);
// prints us per launch for tilings (MT, NT, KW) and the diagnostic variants
// VAR 1 (no activation loads) / 2 (no weight loads).
#include "../qwen3-asr.cpp_amd/csrc/gemm_skinny.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qasr;

struct Shape { const char *name; int N, K, epi; };

__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 1000) p[0] = 1;
}

template <int MT, int NT, int KW, int EPI, int VAR, int CPW = 0>
static double time_cfg(GemmArgs g, const std::vector<uint16_t *> &ws, hipStream_t s, const char *tag) {
    const int NREP = 64;
    dim3 grid(g.N / (16 * NT), (g.M + 16 * MT - 1) / (16 * MT));
    hipGraph_t graph; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < NREP; r++) {
        g.W = ws[r % ws.size()];
        hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, EPI, VAR, CPW>), grid, dim3(64 * KW), 0, s, g);
    }
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(a, s)); CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    const double us = best * 1e3 / NREP;
    const double bytes = (double)g.N * g.K * 2;
    // checksum of the last launch's output (same weights copy for every variant)
    const size_t no = (size_t)g.M * (EPI == EPI_SWIGLU_F16 ? g.N / 2 : g.N);
    double cs = 0;
    if (EPI == EPI_SWIGLU_F16) {
        std::vector<_Float16> h(no); CK(hipMemcpy(h.data(), g.out_f16, no * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < no; i++) cs += (double)h[i] * (double)((i % 97) + 1);
    } else {
        std::vector<float> h(no); CK(hipMemcpy(h.data(), g.out_f32, no * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < no; i++) cs += (double)h[i] * (double)((i % 97) + 1);
    }
    printf("  %-28s MT%d NT%d KW%d VAR%d CPW%d  %7.2f us  %6.0f GB/s  grid %4dx%d  sum %.9g\n", tag, MT, NT, KW, VAR, CPW, us, bytes / us * 1e-3, grid.x,
           grid.y, cs);
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(graph));
    return us;
}

int main(int argc, char **argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 64;
    hipStream_t s; CK(hipStreamCreate(&s));
    Shape shapes[] = {{"qkv 4096x1024", 4096, 1024, EPI_F32}, {"o 1024x2048", 1024, 2048, EPI_F32},
                      {"gu 6144x1024 swiglu", 6144, 1024, EPI_SWIGLU_F16}, {"down 1024x3072", 1024, 3072, EPI_F32}};
    uint16_t *A; float *out, *res; uint16_t *out16;
    CK(hipMalloc(&A, (size_t)128 * 4096 * 2));
    {
        std::vector<_Float16> h((size_t)128 * 4096);
        unsigned x = 777u;
        for (auto &v : h) { x = x * 1664525u + 1013904223u; v = (_Float16)(((x >> 9) * (1.0f / 8388608.0f)) - 0.5f); }
        CK(hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&out, (size_t)128 * 8192 * 4)); CK(hipMalloc(&res, (size_t)128 * 8192 * 4)); CK(hipMalloc(&out16, (size_t)128 * 8192 * 2));
    CK(hipMemset(res, 0, (size_t)128 * 8192 * 4));
    printf("M = %d\n", M);
    {   // the graph's per-launch floor: an empty kernel of 256 workgroups, 64 dependent launches
        hipGraph_t graph; hipGraphExec_t ex;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int r = 0; r < 64; r++) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(512), 0, s, nullptr);
        CK(hipStreamEndCapture(s, &graph));
        CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
        float best = 1e30f;
        for (int it = 0; it < 5; it++) {
            CK(hipEventRecord(a, s)); CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
        }
        printf("empty kernel (256 x 512 threads) in a graph: %.2f us per launch\n", best * 1e3 / 64);
    }
    for (const Shape &sh : shapes) {
        const size_t wb = (size_t)sh.N * sh.K * 2;
        const int NL = (int)((600ull << 20) / wb) + 1;
        std::vector<uint16_t *> ws(NL);
        for (auto &w : ws) { CK(hipMalloc(&w, wb)); CK(hipMemset(w, 0x22, wb)); }
        GemmArgs g{};
        g.A = A; g.lda = sh.K; g.ldw = sh.K; g.M = M; g.N = sh.N; g.K = sh.K;
        g.out_f32 = out; g.ldo = sh.N; g.res = res; g.ldr = sh.N; g.out_f16 = out16; g.ldo16 = sh.N;
        printf("%s (%zu MB, %d copies)\n", sh.name, wb >> 20, NL);
        if (M > 64 || getenv("SKINNY_ALT")) {   // 65..128 rows (round 5; SKINNY_ALT: the same set at any M): fewer activation re-reads (NT 2) against more row blocks
            if (sh.N == 4096) {
                time_cfg<4, 1, 8, EPI_F32, 4, 1>(g, ws, s, "engine (MT4 NT1 CPW1)");
                time_cfg<4, 2, 8, EPI_F32, 4, 1>(g, ws, s, "MT4 NT2 CPW1");
                time_cfg<2, 2, 8, EPI_F32, 4, 1>(g, ws, s, "MT2 NT2 CPW1");
                time_cfg<4, 4, 8, EPI_F32, 4, 1>(g, ws, s, "MT4 NT4 CPW1");
                time_cfg<2, 4, 8, EPI_F32, 4, 1>(g, ws, s, "MT2 NT4 CPW1");
            } else if (sh.N == 1024 && sh.K == 2048) {
                time_cfg<1, 1, 8, EPI_F32, 4, 2>(g, ws, s, "engine (MT1 NT1 CPW2)");
                time_cfg<2, 1, 8, EPI_F32, 4, 2>(g, ws, s, "MT2 NT1 CPW2");
                time_cfg<2, 2, 8, EPI_F32, 4, 2>(g, ws, s, "MT2 NT2 CPW2");
                time_cfg<1, 2, 8, EPI_F32, 4, 2>(g, ws, s, "MT1 NT2 CPW2");
            } else if (sh.epi == EPI_F32) {   // down: the engine's MT2 NT1 (its LDS chunk images of three chunks a
                // wave exceed the LDS, so the chunk loop); round 6 measured every chunk in registers instead
                // (a kernel form since removed): 10.57 us against 9.10 (profiles/r6/skinny_down_regs_ab.txt)
                time_cfg<2, 1, 8, EPI_F32, 12, 0>(g, ws, s, "engine (MT2 chunk loop, wdef)");
                time_cfg<1, 1, 8, EPI_F32, 12, 3>(g, ws, s, "MT1 NT1 CPW3 (LDS, wdef)");
            } else {
                time_cfg<2, 2, 4, EPI_SWIGLU_F16, 4, 2>(g, ws, s, "engine (MT2 NT2 KW4 CPW2)");
                time_cfg<4, 2, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "MT4 NT2 KW8 CPW1");
                time_cfg<4, 4, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "MT4 NT4 KW8 CPW1");
                time_cfg<2, 4, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "MT2 NT4 KW8 CPW1");
                time_cfg<2, 2, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "MT2 NT2 KW8 CPW1");
            }
        } else if (sh.N == 4096) {   // QKV: the engine's <4,1,8> with all chunks in flight (K = 1024: 1 chunk a wave)
            time_cfg<4, 1, 8, EPI_F32, 4, 1>(g, ws, s, "engine (CPW 1)");
            time_cfg<4, 1, 8, EPI_F32, 3>(g, ws, s, "no loads");
            time_cfg<4, 1, 4, EPI_F32, 4, 2>(g, ws, s, "KW4 CPW2");
            time_cfg<2, 1, 8, EPI_F32, 4, 1>(g, ws, s, "MT2 CPW1");
        } else if (sh.N == 1024 && sh.K == 2048) {   // o-proj: <1,1,8> CPW 2
            time_cfg<1, 1, 8, EPI_F32, 4, 2>(g, ws, s, "engine (CPW 2)");
            time_cfg<1, 1, 8, EPI_F32, 3>(g, ws, s, "no loads");
            time_cfg<2, 1, 8, EPI_F32, 4, 2>(g, ws, s, "MT2 CPW2");
            time_cfg<1, 1, 16, EPI_F32, 4, 1>(g, ws, s, "KW16 CPW1");
        } else if (sh.epi == EPI_F32) {   // down: <1,1,8> CPW 3
            time_cfg<1, 1, 8, EPI_F32, 4, 3>(g, ws, s, "engine (CPW 3)");
            time_cfg<1, 1, 8, EPI_F32, 3>(g, ws, s, "no loads");
            time_cfg<1, 1, 16, EPI_F32, 4, 0>(g, ws, s, "KW16 (1.5 chunks: loop)");
        } else {   // gate/up: <2,2,4> CPW 2
            time_cfg<2, 2, 4, EPI_SWIGLU_F16, 4, 2>(g, ws, s, "engine (CPW 2)");
            time_cfg<2, 2, 4, EPI_SWIGLU_F16, 3>(g, ws, s, "no loads");
            time_cfg<2, 2, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "KW8 CPW1");
            time_cfg<4, 2, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "MT4 KW8 CPW1");
            time_cfg<1, 2, 8, EPI_SWIGLU_F16, 4, 1>(g, ws, s, "MT1 KW8 CPW1");
            time_cfg<4, 2, 4, EPI_SWIGLU_F16, 4, 2>(g, ws, s, "MT4 KW4 CPW2");
        }
        for (auto &w : ws) CK(hipFree(w));
    }
    return 0;
}
