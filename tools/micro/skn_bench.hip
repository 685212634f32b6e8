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

namespace qasr {
// ------------------------------------------------------------ RMS norm fold
// Round-6 experiment, measured and not taken (product: rmsnorm_kernel + the
// skinny GEMM, two launches).  Decode batches (9..128 rows), f16 weights, K = 1024: the layer's RMS norm
// (ggml_rms_norm + ggml_mul, src/text_decoder.cpp:480-485 / :542-545) in the
// GEMM's prologue instead of a launch of its own.  The workgroup's 16 MT rows
// of x (fp32) are normalised with rms_row's arithmetic (the values
// launch_rmsnorm_f16 writes) and rounded to fp16 straight into an LDS image
// (row r's 16-B chunk ch at ch ^ (r & 15), lmhead.hip's layout, so the 16
// rows of a fragment read hit distinct banks); wave w then multiplies K chunk
// w of that image against its weight fragments (requested at entry, before
// the prologue) in gemm_skinny_kernel<MT, NT, 8, EPI, 4, 1>'s order -- the
// same fragments, accumulation order and wave-order reduction, so the outputs
// are bit-identical to the two launches (QKV at 16..128 rows; the <=32-row
// SwiGLU tiling of launch_gemm_skinny splits K over 4 waves, this one over 8).
// Measured (this bench, us per launch group incl. the graph's launch floor):
// faster only at 16 rows (QKV 6.23 -> 5.42), slower from 64 (QKV 8.04 ->
// 10.26, gate/up 12.80 -> 15.83 at 128): every block reads its rows as fp32
// from L2, twice the fp16 copy's bytes, before its MFMAs can start.
struct NormIn { const float *xn; int ldxn; const float *norm_w; float eps; };
template <int MT, int NT, int EPI, int WDEF>
__global__ __launch_bounds__(512) void gemm_skinny_norm_kernel(GemmArgs g, NormIn nn) {
    constexpr int KW = 8, NTILE = MT * NT, ROWS = MT * 16, KN = 1024;
    constexpr int IMG_B = ROWS * KN * 2, RED_B = KW * NTILE * 64 * 16;
    static_assert((IMG_B > RED_B ? IMG_B : RED_B) + 512 <= 160 * 1024, "LDS per workgroup");
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[IMG_B > RED_B ? IMG_B : RED_B];
    uint16_t *xs = reinterpret_cast<uint16_t *>(lds_raw);
    floatx4 (*red)[NTILE][64] = reinterpret_cast<floatx4 (*)[NTILE][64]>(lds_raw);
    __shared__ unsigned long long rmax[64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n0 = blockIdx.x * 16 * NT, m0 = blockIdx.y * ROWS;
    const int M = g.M;
    const int q = lane >> 4, c16 = lane & 15;
    auto img = [&](int row, int k) { return row * KN + ((((k >> 3) ^ (row & 15))) << 3) + (k & 7); };

    // this wave's weight fragments (K chunk wid), requested first: they land under the prologue
    u32x4 wq[NT][4];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const u32x4 *wr = (const u32x4 *)(g.W + (long)(n0 + t * 16 + c16) * g.ldw + q * 8) + wid * 16;
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) wq[t][s4] = WDEF ? wr[4 * s4] : __builtin_nontemporal_load(wr + 4 * s4);
    }
    SkinnyEpi<MT, NT, KW, EPI> epi;
    epi.prefetch(g, m0, n0, tid);

    // prologue: wave wid normalises rows wid + 8 r, RB at a time (all of a batch's loads in flight)
    constexpr int R = ROWS / KW, RB = R % 4 == 0 ? 4 : R % 3 == 0 ? 3 : R % 2 == 0 ? 2 : 1;
    float4 nw[4];
#pragma unroll
    for (int i = 0; i < 4; i++) nw[i] = *(const float4 *)(nn.norm_w + 4 * lane + 256 * i);
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += RB) {
        float4 v[RB][4];
#pragma unroll
        for (int r = 0; r < RB; r++) {
            const int m = m0 + wid + KW * (r0 + r);
            const float *xr = nn.xn + (long)(m < M ? m : 0) * nn.ldxn;
#pragma unroll
            for (int i = 0; i < 4; i++) v[r][i] = *(const float4 *)(xr + 4 * lane + 256 * i);
        }
#pragma unroll
        for (int r = 0; r < RB; r++) {   // rms_row<1024>'s arithmetic
            const int rl = wid + KW * (r0 + r);
            double sd = 0.0;
#pragma unroll
            for (int i = 0; i < 4; i++)
                sd += ((double)fmul_rn(v[r][i].x, v[r][i].x) + (double)fmul_rn(v[r][i].y, v[r][i].y)) +
                      ((double)fmul_rn(v[r][i].z, v[r][i].z) + (double)fmul_rn(v[r][i].w, v[r][i].w));
            sd = wave_sum_d(sd);
            const float mean = (float)(sd / KN);
            const float scale = 1.0f / sqrtf(mean + nn.eps);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uint32_t lo = f_to_u16(fmul_rn(fmul_rn(v[r][i].x, scale), nw[i].x)) |
                              ((uint32_t)f_to_u16(fmul_rn(fmul_rn(v[r][i].y, scale), nw[i].y)) << 16);
                uint32_t hi = f_to_u16(fmul_rn(fmul_rn(v[r][i].z, scale), nw[i].z)) |
                              ((uint32_t)f_to_u16(fmul_rn(fmul_rn(v[r][i].w, scale), nw[i].w)) << 16);
                if (m0 + rl >= M) lo = hi = 0u;   // rows past M: zeros (the LDS-DMA path's zero line)
                *(uint2 *)(xs + img(rl, 4 * lane + 256 * i)) = make_uint2(lo, hi);
            }
        }
    }
    __syncthreads();

    floatx4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NT; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
        for (int i = 0; i < MT; i++) {
            const half8 a8 = *(const half8 *)(xs + img(i * 16 + c16, wid * 128 + 32 * s4 + 8 * q));
#pragma unroll
            for (int j = 0; j < NT; j++)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, __builtin_bit_cast(half8, wq[j][s4]), acc[i][j], 0, 0, 0);
        }
    __syncthreads();   // every wave's image reads done before the reduction reuses the LDS
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NT; j++) red[wid][i * NT + j][lane] = acc[i][j];
    __syncthreads();
    epi.run(g, red, rmax, m0, n0, tid);
}

template <int MT, int NT, int EPI>
static void run_skinny_norm(const GemmArgs &g, const NormIn &nn, hipStream_t s) {
    dim3 grid(g.N / (16 * NT), (g.M + 16 * MT - 1) / (16 * MT));
    if (g.wdef) hipLaunchKernelGGL((gemm_skinny_norm_kernel<MT, NT, EPI, 1>), grid, dim3(512), 0, s, g, nn);
    else hipLaunchKernelGGL((gemm_skinny_norm_kernel<MT, NT, EPI, 0>), grid, dim3(512), 0, s, g, nn);
}

bool launch_gemm_skinny_norm(int epi, const GemmArgs &g, const NormIn &nn, hipStream_t s) {
    if (g.no_skinny || !nn.xn || !nn.norm_w || g.M < 9 || g.M > 128 || g.K != 1024 || nn.ldxn % 4 != 0 || g.ldw % 8 != 0 ||
        g.Wq || g.res)
        return false;
    const int mt = (g.M + 15) / 16;
    switch (epi) {
        case EPI_F32:
            if (g.N % 32 != 0) return false;
            // the tilings of launch_gemm_skinny for K = 1024 at these rows (QKV: one K chunk a wave)
            if (g.M > 64) run_skinny_norm<4, 2, EPI_F32>(g, nn, s);
            else if (mt <= 1) run_skinny_norm<1, 1, EPI_F32>(g, nn, s);
            else if (mt <= 2) run_skinny_norm<2, 1, EPI_F32>(g, nn, s);
            else if (mt <= 3) run_skinny_norm<3, 1, EPI_F32>(g, nn, s);
            else run_skinny_norm<4, 1, EPI_F32>(g, nn, s);
            return true;
        case EPI_SWIGLU_F16:
            if (g.N % 64 != 0) return false;
            if (g.M > 64) run_skinny_norm<4, 4, EPI_SWIGLU_F16>(g, nn, s);
            else if (g.M > 32) run_skinny_norm<4, 2, EPI_SWIGLU_F16>(g, nn, s);
            else run_skinny_norm<2, 2, EPI_SWIGLU_F16>(g, nn, s);
            return true;
        default:
            return false;
    }
}

}  // namespace qasr

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
                    GemmArgs b = g; b.wdef = wd; set_out(b, 1);
                    const NormIn nn{x, H, nw, 1e-6f};
                    t1[wd] = time_graph(s, NREP, [&](int r) {
                        GemmArgs h = b; h.W = ws[r % NL];
                        if (!launch_gemm_skinny_norm(sh.epi, h, nn, s)) { printf("norm declined\n"); exit(1); }
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
