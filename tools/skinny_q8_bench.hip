// skinny_q8_bench.hip -- the decode-batch Q8_0 gate/up GEMM (csrc/gemm_skinny.hip,
// included directly): us per launch of the SwiGLU forms, and the bits of the
// fused-quantisation epilogue (EPI_SWIGLU_Q8) against the fp32 SwiGLU output
// quantised on the host with quantize_q8_rows_kernel's arithmetic.
// Usage: skinny_q8_bench [M]   (weights streamed from HBM: > 256 MiB of copies)
#include "../qwen3-asr.cpp_amd/csrc/gemm_skinny.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qasr;

template <int MT, int NT, int KW, int EPI, int CPW>
static double time_cfg(GemmArgs g, const std::vector<int8_t *> &ws, const std::vector<uint16_t *> &wds, hipStream_t s, const char *tag) {
    const int NREP = 64;
    dim3 grid(g.N / (16 * NT), (g.M + 16 * MT - 1) / (16 * MT));
    hipGraph_t graph; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < NREP; r++) {
        g.Wq = ws[r % ws.size()]; g.Wd = wds[r % ws.size()];
        hipLaunchKernelGGL((gemm_skinny_q8_kernel<MT, NT, KW, EPI, 4, CPW>), grid, dim3(64 * KW), 0, s, g);
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
    const double us = best * 1e3 / NREP, bytes = (double)g.N * g.K * 34 / 32;
    printf("  %-34s MT%d NT%d KW%d CPW%d  %7.2f us  %6.0f GB/s  grid %4dx%d\n", tag, MT, NT, KW, CPW, us, bytes / us * 1e-3, grid.x, grid.y);
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(graph));
    return us;
}

int main(int argc, char **argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 64;
    const int N = 6144, K = 1024, F = N / 2;
    if (M < 1 || M > 128) { printf("M in 1..128\n"); return 1; }
    hipStream_t s; CK(hipStreamCreate(&s));
    // activations: int8 [M][K] + fp32 (fp16-valued) block scales [M][K/32]
    int8_t *Aq, *oq; float *Ad, *o32, *od;
    CK(hipMalloc(&Aq, (size_t)128 * K)); CK(hipMalloc(&Ad, (size_t)128 * (K / 32) * 4));
    CK(hipMalloc(&o32, (size_t)128 * F * 4)); CK(hipMalloc(&oq, (size_t)128 * F)); CK(hipMalloc(&od, (size_t)128 * (F / 32) * 4));
    unsigned x = 4321u;
    auto rnd = [&] { x = x * 1664525u + 1013904223u; return x >> 8; };
    {
        std::vector<int8_t> q((size_t)128 * K);
        for (auto &v : q) v = (int8_t)((int)(rnd() % 255) - 127);
        std::vector<float> d((size_t)128 * (K / 32));
        for (auto &v : d) v = (float)(_Float16)(0.002f + 0.0001f * (float)(rnd() % 100));
        CK(hipMemcpy(Aq, q.data(), q.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(Ad, d.data(), d.size() * 4, hipMemcpyHostToDevice));
    }
    const size_t wb = (size_t)N * K;
    const int NL = (int)((600ull << 20) / wb) + 1;
    std::vector<int8_t *> ws(NL);
    std::vector<uint16_t *> wds(NL);
    {
        std::vector<int8_t> q(wb);
        for (auto &v : q) v = (int8_t)((int)(rnd() % 255) - 127);
        std::vector<uint16_t> d((size_t)N * (K / 32));
        for (auto &v : d) { _Float16 h = (_Float16)(0.001f + 0.00005f * (float)(rnd() % 100)); memcpy(&v, &h, 2); }
        for (int i = 0; i < NL; i++) {
            CK(hipMalloc(&ws[i], wb)); CK(hipMalloc(&wds[i], d.size() * 2));
            CK(hipMemcpy(ws[i], q.data(), wb, hipMemcpyHostToDevice));
            CK(hipMemcpy(wds[i], d.data(), d.size() * 2, hipMemcpyHostToDevice));
        }
    }
    GemmArgs g{};
    g.Aq = Aq; g.lda = K; g.Ad = Ad; g.ldad = K / 32; g.ldw = K; g.M = M; g.N = N; g.K = K;
    g.out_f32 = o32; g.ldo = F; g.out_q = oq; g.out_d = od; g.ldoq = F; g.skinny_inflight = 1;
    printf("M = %d, gate/up %dx%d Q8_0 (%d copies)\n", M, N, K, NL);
    // bits: the fused epilogue against the fp32 output quantised on the host
    {
        GemmArgs g1 = g; g1.Wq = ws[0]; g1.Wd = wds[0];
        CK(hipMemset(oq, 0x55, (size_t)128 * F)); CK(hipMemset(od, 0x55, (size_t)128 * (F / 32) * 4));
        // the engine's tiling (K over 8 waves) and the fp32 form with the same K split
        hipLaunchKernelGGL((gemm_skinny_q8_kernel<2, 2, 8, EPI_SWIGLU_F32, 4, 1>), dim3(N / 32, (M + 31) / 32), dim3(512), 0, s, g1);
        hipLaunchKernelGGL((gemm_skinny_q8_kernel<2, 4, 8, EPI_SWIGLU_Q8, 4, 1>), dim3(N / 64, (M + 31) / 32), dim3(512), 0, s, g1);
        CK(hipStreamSynchronize(s));
        std::vector<float> v((size_t)M * F), d((size_t)M * (F / 32));
        std::vector<int8_t> q((size_t)M * F);
        CK(hipMemcpy(v.data(), o32, v.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(q.data(), oq, q.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(d.data(), od, d.size() * 4, hipMemcpyDeviceToHost));
        long bad = 0;
        for (int r = 0; r < M; r++)
            for (int b = 0; b < F / 32; b++) {
                float am = 0.f;
                for (int i = 0; i < 32; i++) am = fmaxf(am, fabsf(v[(size_t)r * F + 32 * b + i]));
                const float dd = (float)(_Float16)(am / 127.f), id = am != 0.f ? 127.f / am : 0.f;
                if (memcmp(&dd, &d[(size_t)r * (F / 32) + b], 4)) bad++;
                for (int i = 0; i < 32; i++)
                    if ((int8_t)rintf(v[(size_t)r * F + 32 * b + i] * id) != q[(size_t)r * F + 32 * b + i]) bad++;
            }
        printf("  EPI_SWIGLU_Q8 vs EPI_SWIGLU_F32 + host quantisation: %ld mismatches %s\n", bad, bad ? "BAD" : "ok");
    }
    time_cfg<2, 2, 4, EPI_SWIGLU_F32, 2>(g, ws, wds, s, "round 5 (f32 out, + quantize)");
    time_cfg<2, 4, 4, EPI_SWIGLU_Q8, 2>(g, ws, wds, s, "fused q8 MT2 NT4 KW4");
    time_cfg<1, 4, 4, EPI_SWIGLU_Q8, 2>(g, ws, wds, s, "fused q8 MT1 NT4 KW4");
    time_cfg<2, 4, 8, EPI_SWIGLU_Q8, 1>(g, ws, wds, s, "engine (fused q8 MT2 NT4 KW8)");
    time_cfg<1, 4, 8, EPI_SWIGLU_Q8, 1>(g, ws, wds, s, "fused q8 MT1 NT4 KW8");
    time_cfg<4, 4, 8, EPI_SWIGLU_Q8, 1>(g, ws, wds, s, "fused q8 MT4 NT4 KW8");
    time_cfg<2, 8, 4, EPI_SWIGLU_Q8, 2>(g, ws, wds, s, "fused q8 MT2 NT8 KW4");
    for (int w = 0; w < NL; w++) { CK(hipFree(ws[w])); CK(hipFree(wds[w])); }
    // the fp32-output projections (QKV, o, down): the engine's tilings and alternatives
    struct Sh { const char *name; int N, K; };
    const Sh shs[] = {{"qkv 4096x1024", 4096, 1024}, {"o 1024x2048", 1024, 2048}, {"down 1024x3072", 1024, 3072}};
    float *res; int8_t *A2; float *Ad2;
    CK(hipMalloc(&res, (size_t)128 * 4096 * 4)); CK(hipMemset(res, 0, (size_t)128 * 4096 * 4));
    CK(hipMalloc(&A2, (size_t)128 * 3072)); CK(hipMemset(A2, 0x13, (size_t)128 * 3072));
    CK(hipMalloc(&Ad2, (size_t)128 * 96 * 4)); CK(hipMemset(Ad2, 0x3a, (size_t)128 * 96 * 4));
    CK(hipFree(o32)); CK(hipMalloc(&o32, (size_t)128 * 4096 * 4));
    for (const Sh &sh : shs) {
        const size_t wb2 = (size_t)sh.N * sh.K;
        const int NL2 = (int)((600ull << 20) / wb2) + 1;
        std::vector<int8_t *> w2(NL2);
        std::vector<uint16_t *> d2(NL2);
        for (int i = 0; i < NL2; i++) {
            CK(hipMalloc(&w2[i], wb2)); CK(hipMemset(w2[i], 0x21, wb2));
            CK(hipMalloc(&d2[i], wb2 / 16)); CK(hipMemset(d2[i], 0x11, wb2 / 16));
        }
        GemmArgs h{};
        h.Aq = A2; h.lda = sh.K; h.Ad = Ad2; h.ldad = sh.K / 32; h.ldw = sh.K; h.M = M; h.N = sh.N; h.K = sh.K;
        h.out_f32 = o32; h.ldo = sh.N; h.res = res; h.ldr = sh.N; h.skinny_inflight = 1;
        printf("%s (%d copies)\n", sh.name, NL2);
        if (sh.N == 4096) {
            time_cfg<2, 1, 8, EPI_F32, 1>(h, w2, d2, s, "engine (MT2 NT1 KW8)");
            time_cfg<4, 1, 8, EPI_F32, 1>(h, w2, d2, s, "MT4 NT1 KW8");
            time_cfg<2, 2, 8, EPI_F32, 1>(h, w2, d2, s, "MT2 NT2 KW8");
            time_cfg<4, 2, 8, EPI_F32, 1>(h, w2, d2, s, "MT4 NT2 KW8");
            time_cfg<2, 1, 4, EPI_F32, 2>(h, w2, d2, s, "MT2 NT1 KW4");
        } else if (sh.K == 2048) {
            time_cfg<1, 1, 8, EPI_F32, 2>(h, w2, d2, s, "engine (MT1 NT1 KW8)");
            time_cfg<2, 1, 8, EPI_F32, 2>(h, w2, d2, s, "MT2 NT1 KW8");
            time_cfg<4, 1, 8, EPI_F32, 2>(h, w2, d2, s, "MT4 NT1 KW8");
            time_cfg<1, 1, 16, EPI_F32, 1>(h, w2, d2, s, "MT1 NT1 KW16");
            time_cfg<2, 1, 16, EPI_F32, 1>(h, w2, d2, s, "MT2 NT1 KW16");
        } else {
            time_cfg<1, 1, 8, EPI_F32, 3>(h, w2, d2, s, "engine (MT1 NT1 KW8)");
            time_cfg<2, 1, 8, EPI_F32, 3>(h, w2, d2, s, "MT2 NT1 KW8");
            time_cfg<2, 1, 12, EPI_F32, 2>(h, w2, d2, s, "MT2 NT1 KW12");
        }
        for (int i = 0; i < NL2; i++) { CK(hipFree(w2[i])); CK(hipFree(d2[i])); }
    }
    return 0;
}
