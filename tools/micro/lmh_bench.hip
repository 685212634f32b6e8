// lmh_bench.hip -- the decode-batch LM head: separate launches (RMS norm ->
// fp16 rows, key reset, gemm_skinny_kernel<4,4,2> ARGMAX, step advance,
// argmax finish) against lmhead.hip's one launch, at M = 64 / 48 / 32 / 16 / 9.
// Checks: logits bit-identical, token ids equal, bookkeeping (pos, n_kv, step,
// hist) equal, amax / done back to zero.  Times: hipGraph of NREP steps over two
// weight copies (2 x 311 MB > the 256 MB Infinity Cache: weights from HBM).
#include "../../qwen3-asr.cpp_amd/csrc/gemm_skinny.hip"
#include "../../qwen3-asr.cpp_amd/csrc/lmhead.hip"
#include "../../qwen3-asr.cpp_amd/csrc/elementwise.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qasr;

__global__ void fill_rand_f16(uint16_t *p, long n, uint32_t seed, float amp) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        p[i] = __builtin_bit_cast(uint16_t, (_Float16)(((x >> 8) * (1.0f / 16777216.0f) - 0.5f) * amp));
    }
}

struct Bufs {
    float *x, *normw, *logits; uint16_t *xh;
    unsigned long long *amax; unsigned int *done; int *tok, *hist, *step, *pos, *nkv;
};

static void old_step(const Bufs &b, const uint16_t *W, int M, int N, bool logits, hipStream_t s) {
    launch_fill_u64(b.amax, M, 0ull, s);
    launch_rmsnorm_f16(b.x, 1024, nullptr, M, 1024, b.normw, 1e-6f, b.xh, s);
    GemmArgs g{};
    g.A = b.xh; g.lda = 1024; g.W = W; g.ldw = 1024; g.M = M; g.N = N; g.K = 1024;
    g.out_f32 = logits ? b.logits : nullptr; g.ldo = N; g.amax = b.amax;
    if (!launch_gemm_skinny(EPI_ARGMAX, g, s)) { printf("skinny declined\n"); exit(1); }
    launch_step_advance(b.pos, b.nkv, b.step, M, s);
    launch_argmax_finish(b.amax, M, b.tok, b.hist, 64, b.step, s);
    launch_fill_u64(b.amax, M, 0ull, s);
}

static void new_step(const Bufs &b, const uint16_t *W, int M, int N, bool logits, hipStream_t s) {
    GemvArgs g{};
    g.x = b.x; g.ldx = 1024; g.norm_w = b.normw; g.eps = 1e-6f; g.W = W; g.K = 1024; g.N = N; g.M = M;
    g.out_f32 = logits ? b.logits : nullptr; g.ldo = N; g.amax = b.amax; g.done = b.done; g.tok_out = b.tok;
    g.hist = b.hist; g.hist_stride = 64; g.step = b.step; g.pos = b.pos; g.nkv = b.nkv;
    if (!launch_lmhead_batch(g, s)) { printf("lmhead declined\n"); exit(1); }
}

static void reset_state(const Bufs &b) {
    CK(hipMemset(b.amax, 0, 64 * 8)); CK(hipMemset(b.done, 0, 4)); CK(hipMemset(b.tok, 0, 64 * 4));
    CK(hipMemset(b.hist, 0xff, 64 * 64 * 4)); CK(hipMemset(b.step, 0, 4)); CK(hipMemset(b.pos, 0, 64 * 4));
    CK(hipMemset(b.nkv, 0, 64 * 4));
}

template <typename F>
static double time_graph(F step, const std::vector<uint16_t *> &ws, hipStream_t s) {
    const int NREP = 32;
    hipGraph_t graph; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < NREP; r++) step(ws[r % ws.size()]);
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
    hipEvent_t a, e; CK(hipEventCreate(&a)); CK(hipEventCreate(&e));
    CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(a, s)); CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(e, s)); CK(hipEventSynchronize(e));
        float ms; CK(hipEventElapsedTime(&ms, a, e)); best = ms < best ? ms : best;
    }
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(graph));
    return best * 1e3 / NREP;
}

template <int MT, int WPG, int D>
static void variant(const Bufs &b, const std::vector<uint16_t *> &ws, int M, int N, hipStream_t s) {
    (void)hipFuncSetAttribute((const void *)lmhead_batch_kernel<MT, WPG, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MT * 16 * 1024 * 2);
    GemvArgs g{};
    g.x = b.x; g.ldx = 1024; g.norm_w = b.normw; g.eps = 1e-6f; g.K = 1024; g.N = N; g.M = M;
    g.amax = b.amax; g.done = b.done; g.tok_out = b.tok;
    g.hist = b.hist; g.hist_stride = 64; g.step = b.step; g.pos = b.pos; g.nkv = b.nkv;
    const double t = time_graph([&](const uint16_t *W) {
        g.W = W;
        hipLaunchKernelGGL((lmhead_batch_kernel<MT, WPG, D>), dim3(256), dim3(64 * WPG), MT * 16 * 1024 * 2, s, g);
    }, ws, s);
    printf("  M=%d MT%d WPG%2d D%d  %7.2f us  %.3f of 8 TB/s\n", M, MT, WPG, D, t, (double)N * 2048 / t * 1e-3 / 8000.0);
}

int main() {
    const int N = 151936;
    hipStream_t s; CK(hipStreamCreate(&s));
    std::vector<uint16_t *> ws(2);
    const size_t wb = (size_t)N * 1024 * 2;
    for (int i = 0; i < 2; i++) {
        CK(hipMalloc(&ws[i], wb));
        hipLaunchKernelGGL(fill_rand_f16, dim3(4096), dim3(256), 0, s, ws[i], (long)N * 1024, 1234u + i, 0.25f);
    }
    Bufs b{};
    CK(hipMalloc(&b.x, 64 * 1024 * 4)); CK(hipMalloc(&b.normw, 1024 * 4)); CK(hipMalloc(&b.logits, (size_t)64 * N * 4));
    CK(hipMalloc(&b.xh, 64 * 1024 * 2)); CK(hipMalloc(&b.amax, 64 * 8)); CK(hipMalloc(&b.done, 4));
    CK(hipMalloc(&b.tok, 64 * 4)); CK(hipMalloc(&b.hist, 64 * 64 * 4)); CK(hipMalloc(&b.step, 4));
    CK(hipMalloc(&b.pos, 64 * 4)); CK(hipMalloc(&b.nkv, 64 * 4));
    {
        std::vector<float> hx(64 * 1024), hw(1024);
        unsigned x = 99u;
        for (auto &v : hx) { x = x * 1664525u + 1013904223u; v = ((x >> 9) * (1.0f / 8388608.0f) - 0.5f) * 4.0f; }
        for (auto &v : hw) { x = x * 1664525u + 1013904223u; v = 0.5f + (x >> 9) * (1.0f / 8388608.0f); }
        CK(hipMemcpy(b.x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(b.normw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    }
    CK(hipStreamSynchronize(s));
    int bad = 0;
    for (int M : {64, 48, 33, 32, 16, 9}) {
        std::vector<float> lo((size_t)M * N), ln((size_t)M * N);
        std::vector<int> to(64), tn(64), ho(64 * 64), hn(64 * 64), po(64), pn(64), ko(64), kn(64);
        int so = 0, sn = 0;
        reset_state(b);
        old_step(b, ws[0], M, N, true, s); old_step(b, ws[0], M, N, true, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(lo.data(), b.logits, lo.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(to.data(), b.tok, 256, hipMemcpyDeviceToHost)); CK(hipMemcpy(ho.data(), b.hist, 64 * 64 * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(po.data(), b.pos, 256, hipMemcpyDeviceToHost)); CK(hipMemcpy(ko.data(), b.nkv, 256, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&so, b.step, 4, hipMemcpyDeviceToHost));
        CK(hipMemset(b.logits, 0, (size_t)64 * N * 4));
        reset_state(b);
        new_step(b, ws[0], M, N, true, s); new_step(b, ws[0], M, N, true, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(ln.data(), b.logits, ln.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(tn.data(), b.tok, 256, hipMemcpyDeviceToHost)); CK(hipMemcpy(hn.data(), b.hist, 64 * 64 * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pn.data(), b.pos, 256, hipMemcpyDeviceToHost)); CK(hipMemcpy(kn.data(), b.nkv, 256, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&sn, b.step, 4, hipMemcpyDeviceToHost));
        unsigned long long am[64]; unsigned dn = 7;
        CK(hipMemcpy(am, b.amax, 64 * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&dn, b.done, 4, hipMemcpyDeviceToHost));
        const bool lg_eq = memcmp(lo.data(), ln.data(), lo.size() * 4) == 0;
        bool ok = lg_eq && memcmp(to.data(), tn.data(), M * 4) == 0 && memcmp(ho.data(), hn.data(), sizeof(int) * 64 * 64) == 0 &&
                  memcmp(po.data(), pn.data(), M * 4) == 0 && memcmp(ko.data(), kn.data(), M * 4) == 0 && so == sn && dn == 0;
        for (int i = 0; i < M; i++) ok = ok && am[i] == 0;
        // host argmax of the new logits (first index) equals the token
        for (int m = 0; m < M; m++) {
            int bi = 0;
            for (int n = 1; n < N; n++) if (ln[(size_t)m * N + n] > ln[(size_t)m * N + bi]) bi = n;
            ok = ok && bi == tn[m];
        }
        long ndiff = 0;
        for (size_t i = 0; i < lo.size(); i++) ndiff += lo[i] != ln[i];
        const double t_old = time_graph([&](const uint16_t *W) { old_step(b, W, M, N, false, s); }, ws, s);
        const double t_new = time_graph([&](const uint16_t *W) { new_step(b, W, M, N, false, s); }, ws, s);
        printf("M=%2d  separate %7.2f us  one launch %7.2f us (%6.0f GB/s, %.3f of 8 TB/s)  logits %s (%ld differ)  tok0 %d step %d  %s\n", M,
               t_old, t_new, wb / t_new * 1e-3, wb / t_new * 1e-3 / 8000.0, lg_eq ? "bit-identical" : "DIFFER", ndiff, tn[0], sn,
               ok ? "OK" : "MISMATCH");
        bad += !ok;
    }
    reset_state(b);
    variant<4, 8, 4>(b, ws, 64, N, s);
    variant<4, 8, 6>(b, ws, 64, N, s);
    variant<4, 8, 8>(b, ws, 64, N, s);
    variant<4, 4, 8>(b, ws, 64, N, s);
    variant<4, 4, 12>(b, ws, 64, N, s);
    variant<1, 16, 3>(b, ws, 16, N, s);
    variant<1, 8, 4>(b, ws, 16, N, s);
    variant<1, 8, 8>(b, ws, 16, N, s);
    variant<2, 8, 8>(b, ws, 32, N, s);
    return bad ? 1 : 0;
}
