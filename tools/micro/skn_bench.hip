// skn_bench.hip -- decode-batch projections at 16..128 rows (round 6):
//  * the RMS norm folded into the QKV / gate-up skinny GEMM's prologue
//    (launch_gemm_skinny_norm) against the two launches it replaces
//    (rmsnorm_kernel's arithmetic + launch_gemm_skinny), bit for bit;
//  * the skinny GEMMs' weights with the default cache policy (GemmArgs::wdef)
//    against nontemporal loads (o / down at 65..128 rows read each weight
//    tile once per 32-row block).
// Each variant: a hipGraph of NREP dependent launches over NL weight copies
// (> 256 MiB Infinity Cache, so weights stream from HBM as in a decode step);
// us per launch group.  Build: see tools/r6/skn.sh.
#include "../../qwen3-asr.cpp_amd/csrc/gemm_skinny.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qasr;

// rmsnorm_kernel<1024> (elementwise.hip): one wave per row, rms_row's arithmetic
__global__ __launch_bounds__(256) void norm_ref(const float *x, int ldx, int M, const float *w, float eps, uint16_t *y) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    float4 v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = *(const float4 *)(x + (long)row * ldx + 4 * lane + 256 * i);
    rms_row<1024>(v, w, eps, row, y, nullptr, nullptr, nullptr);
}

static double time_graph(hipStream_t s, int nrep, const std::function<void(int)> &enq) {
    hipGraph_t graph;
    hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < nrep; r++) enq(r);
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int it = 0; it < 7; it++) {
        CK(hipEventRecord(a, s)); CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(graph));
    return best * 1e3 / nrep;
}

template <class T>
static std::vector<T> dl(const T *p, size_t n) {
    std::vector<T> h(n);
    CK(hipMemcpy(h.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
    return h;
}

int main(int argc, char **argv) {
    hipStream_t s; CK(hipStreamCreate(&s));
    const int H = 1024, NREP = 64;
    float *x, *nw, *out0, *out1, *res;
    uint16_t *xh, *o16a, *o16b;
    CK(hipMalloc(&x, (size_t)128 * H * 4)); CK(hipMalloc(&nw, H * 4)); CK(hipMalloc(&xh, (size_t)128 * 4096 * 2));
    CK(hipMalloc(&out0, (size_t)128 * 8192 * 4)); CK(hipMalloc(&out1, (size_t)128 * 8192 * 4)); CK(hipMalloc(&res, (size_t)128 * 8192 * 4));
    CK(hipMalloc(&o16a, (size_t)128 * 8192 * 2)); CK(hipMalloc(&o16b, (size_t)128 * 8192 * 2));
    {
        std::vector<float> hx((size_t)128 * H), hw(H);
        unsigned st = 4242u;
        auto fr = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 9) * (1.0f / 8388608.0f)) - 0.5f; };
        for (auto &v : hx) v = 4.0f * fr();
        for (auto &v : hw) v = 1.0f + 0.5f * fr();
        CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(nw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
        std::vector<_Float16> ha((size_t)128 * 4096);
        for (auto &v : ha) v = (_Float16)fr();
        CK(hipMemcpy(xh, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemset(res, 0, (size_t)128 * 8192 * 4));
    }
    struct Shape { const char *name; int N, K, epi; bool norm; };
    Shape shapes[] = {{"qkv 4096x1024 (+norm)", 4096, 1024, EPI_F32, true}, {"gu 6144x1024 swiglu (+norm)", 6144, 1024, EPI_SWIGLU_F16, true},
                      {"o 1024x2048 +res", 1024, 2048, EPI_F32, false}, {"down 1024x3072 +res", 1024, 3072, EPI_F32, false}};
    int Ms[] = {16, 64, 100, 128};
    for (const Shape &sh : shapes) {
        const size_t wb = (size_t)sh.N * sh.K * 2;
        const int NL = (int)((600ull << 20) / wb) + 1;
        std::vector<uint16_t *> ws(NL);
        for (auto &w : ws) {
            CK(hipMalloc(&w, wb));
            std::vector<_Float16> hw(wb / 2);
            unsigned st = 99u + (unsigned)(&w - &ws[0]);
            for (auto &v : hw) { st = st * 1664525u + 1013904223u; v = (_Float16)(((st >> 9) * (1.0f / 8388608.0f) - 0.5f) * 0.05f); }
            CK(hipMemcpy(w, hw.data(), wb, hipMemcpyHostToDevice));
        }
        printf("%s (%zu MB, %d copies)\n", sh.name, wb >> 20, NL);
        for (int M : Ms) {
            GemmArgs g{};
            g.M = M; g.N = sh.N; g.K = sh.K; g.ldw = sh.K; g.skinny_inflight = 1;
            const bool swi = sh.epi == EPI_SWIGLU_F16;
            const size_t no = (size_t)M * (swi ? sh.N / 2 : sh.N);
            auto set_out = [&](GemmArgs &h, int which) {
                if (swi) { h.out_f16 = which ? o16b : o16a; h.ldo16 = sh.N / 2; }
                else { h.out_f32 = which ? out1 : out0; h.ldo = sh.N; }
                if (!sh.norm) { h.res = res; h.ldr = sh.N; }
            };
            auto cmp = [&]() -> long {
                long d = 0;
                if (swi) { auto a = dl(o16a, no), b = dl(o16b, no); for (size_t i = 0; i < no; i++) d += a[i] != b[i]; }
                else { auto a = dl(out0, no), b = dl(out1, no); for (size_t i = 0; i < no; i++) d += memcmp(&a[i], &b[i], 4) != 0; }
                return d;
            };
            if (sh.norm) {
                double t2[2], t1[2];
                for (int wd = 0; wd < 2; wd++) {
                    GemmArgs a = g; a.A = xh; a.lda = H; a.wdef = wd; set_out(a, 0);
                    t2[wd] = time_graph(s, NREP, [&](int r) {
                        GemmArgs h = a; h.W = ws[r % NL];
                        hipLaunchKernelGGL(norm_ref, dim3((M + 3) / 4), dim3(256), 0, s, x, H, M, nw, 1e-6f, xh);
                        if (!launch_gemm_skinny(sh.epi, h, s)) { printf("skinny declined\n"); exit(1); }
                    });
                    GemmArgs b = g; b.xn = x; b.ldxn = H; b.norm_w = nw; b.eps = 1e-6f; b.wdef = wd; set_out(b, 1);
                    t1[wd] = time_graph(s, NREP, [&](int r) {
                        GemmArgs h = b; h.W = ws[r % NL];
                        if (!launch_gemm_skinny_norm(sh.epi, h, s)) { printf("norm declined\n"); exit(1); }
                    });
                }
                // same weights copy for both: the last launch of each graph used ws[(NREP - 1) % NL]
                printf("  M %3d  norm + skinny %6.2f / %6.2f us (nt / default policy)   fused %6.2f / %6.2f us   outputs differ: %ld of %zu\n",
                       M, t2[0], t2[1], t1[0], t1[1], cmp(), no);
            } else {
                double t[2];
                for (int wd = 0; wd < 2; wd++) {
                    GemmArgs a = g; a.A = xh; a.lda = sh.K; a.wdef = wd; set_out(a, wd);
                    t[wd] = time_graph(s, NREP, [&](int r) {
                        GemmArgs h = a; h.W = ws[r % NL];
                        if (!launch_gemm_skinny(sh.epi, h, s)) { printf("skinny declined\n"); exit(1); }
                    });
                }
                printf("  M %3d  skinny %6.2f us (nt)  %6.2f us (default policy)   outputs differ: %ld of %zu\n", M, t[0], t[1], cmp(), no);
            }
        }
        for (auto &w : ws) CK(hipFree(w));
    }
    return 0;
}
