// lmh128_bench.hip -- the decode-batch LM head at 65..128 rows: the round-5
// form (one lmhead_batch_kernel launch per 64-row half, each streaming the
// whole 311 MB embedding) against lmhead.hip's lmhead128_kernel (rows in
// registers, the embedding read once).  Checks: logits bit-identical, token
// ids equal, bookkeeping (pos, n_kv, step, hist) equal, amax / done back to
// zero.  Times: hipGraph of NREP steps over two weight copies (2 x 311 MB >
// the 256 MB Infinity Cache: weights from HBM).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../include
//        -I../../qwen3-asr.cpp_amd/csrc lmh128_bench.hip -o lmh128_bench
#include "../../qwen3-asr.cpp_amd/csrc/lmhead.hip"

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

constexpr int MR = 128, HS = 64;   // rows at most, hist stride
struct Bufs {
    float *x, *normw, *logits;
    unsigned long long *amax; unsigned int *done; int *tok, *hist, *step, *pos, *nkv;
};

static GemvArgs args(const Bufs &b, const uint16_t *W, int M, int N, bool logits) {
    GemvArgs g{};
    g.x = b.x; g.ldx = 1024; g.norm_w = b.normw; g.eps = 1e-6f; g.W = W; g.K = 1024; g.N = N; g.M = M;
    g.out_f32 = logits ? b.logits : nullptr; g.ldo = N; g.amax = b.amax; g.done = b.done; g.tok_out = b.tok;
    g.hist = b.hist; g.hist_stride = HS; g.step = b.step; g.pos = b.pos; g.nkv = b.nkv;
    return g;
}
// the round-5 path: one launch per 64-row half, the first leaving the step counter to the second
static void old_step(const Bufs &b, const uint16_t *W, int M, int N, bool logits, hipStream_t s) {
    const GemvArgs g = args(b, W, M, N, logits);
    GemvArgs a = g;
    a.M = 64;
    a.keep_step = 1;
    run_lmhead<4>(a, s);
    GemvArgs c = g;
    c.M = M - 64;
    c.x = g.x + (long)64 * g.ldx;
    if (g.out_f32) c.out_f32 = g.out_f32 + (long)64 * g.ldo;
    c.amax = g.amax + 64;
    c.tok_out = g.tok_out + 64;
    c.hist = g.hist + (long)64 * g.hist_stride;
    c.pos = g.pos + 64;
    c.nkv = g.nkv + 64;
    c.keep_step = 0;
    const int mt = (c.M + 15) / 16;
    if (mt == 1) run_lmhead<1>(c, s);
    else if (mt == 2) run_lmhead<2>(c, s);
    else if (mt == 3) run_lmhead<3>(c, s);
    else run_lmhead<4>(c, s);
}
static void new_step(const Bufs &b, const uint16_t *W, int M, int N, bool logits, hipStream_t s) {
    if (!launch_lmhead_batch(args(b, W, M, N, logits), s)) { printf("lmhead declined\n"); exit(1); }
}

static void reset_state(const Bufs &b) {
    CK(hipMemset(b.amax, 0, MR * 8)); CK(hipMemset(b.done, 0, 4)); CK(hipMemset(b.tok, 0, MR * 4));
    CK(hipMemset(b.hist, 0xff, MR * HS * 4)); CK(hipMemset(b.step, 0, 4)); CK(hipMemset(b.pos, 0, MR * 4));
    CK(hipMemset(b.nkv, 0, MR * 4));
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
    CK(hipMalloc(&b.x, MR * 1024 * 4)); CK(hipMalloc(&b.normw, 1024 * 4)); CK(hipMalloc(&b.logits, (size_t)MR * N * 4));
    CK(hipMalloc(&b.amax, MR * 8)); CK(hipMalloc(&b.done, 4));
    CK(hipMalloc(&b.tok, MR * 4)); CK(hipMalloc(&b.hist, MR * HS * 4)); CK(hipMalloc(&b.step, 4));
    CK(hipMalloc(&b.pos, MR * 4)); CK(hipMalloc(&b.nkv, MR * 4));
    {
        std::vector<float> hx(MR * 1024), hw(1024);
        unsigned x = 99u;
        for (auto &v : hx) { x = x * 1664525u + 1013904223u; v = ((x >> 9) * (1.0f / 8388608.0f) - 0.5f) * 4.0f; }
        for (auto &v : hw) { x = x * 1664525u + 1013904223u; v = 0.5f + (x >> 9) * (1.0f / 8388608.0f); }
        CK(hipMemcpy(b.x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(b.normw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    }
    CK(hipStreamSynchronize(s));
    int bad = 0;
    for (int M : {128, 100, 65}) {
        std::vector<float> lo((size_t)M * N), ln((size_t)M * N);
        std::vector<int> to(MR), tn(MR), ho(MR * HS), hn(MR * HS), po(MR), pn(MR), ko(MR), kn(MR);
        int so = 0, sn = 0;
        reset_state(b);
        old_step(b, ws[0], M, N, true, s); old_step(b, ws[0], M, N, true, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(lo.data(), b.logits, lo.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(to.data(), b.tok, MR * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(ho.data(), b.hist, MR * HS * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(po.data(), b.pos, MR * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(ko.data(), b.nkv, MR * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&so, b.step, 4, hipMemcpyDeviceToHost));
        CK(hipMemset(b.logits, 0, (size_t)MR * N * 4));
        reset_state(b);
        new_step(b, ws[0], M, N, true, s); new_step(b, ws[0], M, N, true, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(ln.data(), b.logits, ln.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(tn.data(), b.tok, MR * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(hn.data(), b.hist, MR * HS * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pn.data(), b.pos, MR * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(kn.data(), b.nkv, MR * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&sn, b.step, 4, hipMemcpyDeviceToHost));
        unsigned long long am[MR]; unsigned dn = 7;
        CK(hipMemcpy(am, b.amax, MR * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&dn, b.done, 4, hipMemcpyDeviceToHost));
        long ndiff = 0;
        for (size_t i = 0; i < lo.size(); i++) ndiff += memcmp(&lo[i], &ln[i], 4) != 0;
        bool ok = ndiff == 0 && memcmp(to.data(), tn.data(), M * 4) == 0 && memcmp(ho.data(), hn.data(), sizeof(int) * MR * HS) == 0 &&
                  memcmp(po.data(), pn.data(), M * 4) == 0 && memcmp(ko.data(), kn.data(), M * 4) == 0 && so == sn && sn == 2 && dn == 0;
        for (int i = 0; i < M; i++) ok = ok && am[i] == 0;
        for (int m = 0; m < M; m++) {   // host argmax of the new logits (first index) equals the token
            int bi = 0;
            for (int n = 1; n < N; n++) if (ln[(size_t)m * N + n] > ln[(size_t)m * N + bi]) bi = n;
            ok = ok && bi == tn[m];
        }
        const double t_old = time_graph([&](const uint16_t *W) { old_step(b, W, M, N, false, s); }, ws, s);
        const double t_new = time_graph([&](const uint16_t *W) { new_step(b, W, M, N, false, s); }, ws, s);
        printf("M=%3d  two launches %7.2f us  one launch %7.2f us (%.2fx, %.3f of 8 TB/s)  logits differ %ld  %s\n", M, t_old, t_new,
               t_old / t_new, (double)N * 2048 / t_new * 1e-3 / 8000.0, ndiff, ok ? "OK" : "MISMATCH");
        bad += !ok;
    }
    printf(bad ? "FAIL\n" : "all equal\n");
    return bad ? 1 : 0;
}
