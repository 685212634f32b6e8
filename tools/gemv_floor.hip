// gemv_floor.hip -- microbenchmark of the batch-1 decode projections.
//
// Times hipGraph-captured chains of dependent launches over NL distinct
// weight sets (NL * bytes > 256 MiB Infinity Cache, so every launch streams
// from HBM as in the real decode step) and reports us per launch:
//   cur     qasr::launch_gemv (libqasr.so)
//   wave    per-wave experimental kernel: no LDS, no block barrier; every
//           wave loads its own x slice (and redoes the RMS norm) next to its
//           weight rows
//   stream  pure weight streaming with the same grid (floor of the shape)
//   empty   empty kernel with the same grid (dispatch floor)
// and the four projections of one decoder layer chained (qkv, o, gate/up,
// down) for cur and wave.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../qwen3-asr.cpp_amd/csrc/dev_common.h"
#include "../qwen3-asr.cpp_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct WArgs {
    const float *x;            // fp32 [K] (NORM) or null
    const uint16_t *xh;        // fp16 [K] (no norm)
    const float *norm_w;
    const uint16_t *W;         // [N(*2 interleaved for SWIGLU)][K]
    const float *res;
    float *out;                // fp32 [N]
    uint16_t *out16;           // fp16 [N] (SWIGLU)
    int N;
    float eps;
};

template <int K, int RPW, bool NORM, bool SWIGLU>
__global__ __launch_bounds__(256) void gemv_wave(WArgs a) {
    constexpr int NT = K / 512;
    constexpr int NR = SWIGLU ? 2 : 1;
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    half8 wv[RPW][NR][NT];
#pragma unroll
    for (int r = 0; r < RPW; r++)
#pragma unroll
        for (int q = 0; q < NR; q++)
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const int o = min(row0 + r, a.N - 1);
                const long wrow = SWIGLU ? 32L * (o >> 4) + (o & 15) + 16 * q : o;
                wv[r][q][t] = __builtin_nontemporal_load((const half8 *)(a.W + wrow * K + t * 512 + lane * 8));
            }
    float xf[NT][8];
    if constexpr (NORM) {
        float4 xv[NT][2];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            xv[t][0] = *(const float4 *)(a.x + t * 512 + lane * 8);
            xv[t][1] = *(const float4 *)(a.x + t * 512 + lane * 8 + 4);
        }
        double ss = 0.0;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const float v[8] = {xv[t][0].x, xv[t][0].y, xv[t][0].z, xv[t][0].w, xv[t][1].x, xv[t][1].y, xv[t][1].z, xv[t][1].w};
#pragma unroll
            for (int e = 0; e < 8; e++) { xf[t][e] = v[e]; ss += (double)(v[e] * v[e]); }
        }
        ss = wave_sum_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / K) + a.eps);
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const float4 w0 = *(const float4 *)(a.norm_w + t * 512 + lane * 8);
            const float4 w1 = *(const float4 *)(a.norm_w + t * 512 + lane * 8 + 4);
            const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
            for (int e = 0; e < 8; e++) xf[t][e] = (float)f2h(fmul_rn(fmul_rn(xf[t][e], scale), w[e]));
        }
    } else {
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const half8 h = *(const half8 *)(a.xh + t * 512 + lane * 8);
#pragma unroll
            for (int e = 0; e < 8; e++) xf[t][e] = (float)h[e];
        }
    }
#pragma unroll
    for (int r = 0; r < RPW; r++) {
        float acc[NR];
#pragma unroll
        for (int q = 0; q < NR; q++) {
            acc[q] = 0.f;
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int e = 0; e < 8; e++) acc[q] = fmaf((float)wv[r][q][t][e], xf[t][e], acc[q]);
            acc[q] = wave_sum(acc[q]);
        }
        const int o = row0 + r;
        if (lane == 0 && o < a.N) {
            if constexpr (SWIGLU) {
                a.out16[o] = f_to_u16(acc[0] / (1.0f + expf(-acc[0])) * acc[1]);
            } else {
                float y = acc[0];
                if (a.res) y = fadd_rn(y, a.res[o]);
                a.out[o] = y;
            }
        }
    }
}

template <int K, int RPW, int NR>
__global__ __launch_bounds__(256) void stream_only(const uint16_t *W, int N, float *out) {
    constexpr int NT = K / 512;
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    float acc = 0.f;
    half8 wv[RPW * NR][NT];
#pragma unroll
    for (int r = 0; r < RPW * NR; r++)
#pragma unroll
        for (int t = 0; t < NT; t++)
            wv[r][t] = __builtin_nontemporal_load((const half8 *)(W + (long)(min(row0 * NR + r, N * NR - 1)) * K + t * 512 + lane * 8));
#pragma unroll
    for (int r = 0; r < RPW * NR; r++)
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int e = 0; e < 8; e++) acc += (float)wv[r][t][e];
    acc = wave_sum(acc);
    if (lane == 0 && row0 < N) out[row0] = acc;
}

__global__ void empty_k(float *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && out[0] == 12345.f) out[1] = 0.f;
}

struct Shape { const char *name; int N, K; bool norm, swiglu; };

static float time_graph(hipStream_t s, int reps, void (*body)(hipStream_t, void *), void *ctx, int launches) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    body(s, ctx);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; r++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return ms * 1e3f / (reps * launches);
}

struct Bufs {
    std::vector<uint16_t *> W;   // per layer
    float *x, *nw, *res, *out;
    uint16_t *xh, *out16;
    int NL;
    Shape sh;
    int variant;   // 0 cur, 1 wave, 2 stream, 3 empty
    int rpw;
};

template <int K, int RPW>
static void launch_wave(const Shape &sh, const WArgs &a, hipStream_t s) {
    const int rows_per_block = 4 * RPW;
    const int grid = (sh.N + rows_per_block - 1) / rows_per_block;
    if (sh.swiglu) hipLaunchKernelGGL((gemv_wave<K, RPW, true, true>), dim3(grid), dim3(256), 0, s, a);
    else if (sh.norm) hipLaunchKernelGGL((gemv_wave<K, RPW, true, false>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((gemv_wave<K, RPW, false, false>), dim3(grid), dim3(256), 0, s, a);
}

template <int K>
static void launch_wave_k(const Shape &sh, const WArgs &a, int rpw, hipStream_t s) {
    if (rpw == 1) launch_wave<K, 1>(sh, a, s);
    else if (rpw == 2) launch_wave<K, 2>(sh, a, s);
    else launch_wave<K, 4>(sh, a, s);
}

template <int K>
static void launch_stream_k(const Shape &sh, const uint16_t *W, float *out, int rpw, hipStream_t s) {
    const int NR = sh.swiglu ? 2 : 1;
    const int grid = (sh.N + 4 * rpw - 1) / (4 * rpw);
    if (rpw == 1) { if (NR == 2) hipLaunchKernelGGL((stream_only<K, 1, 2>), dim3(grid), dim3(256), 0, s, W, sh.N, out);
                    else hipLaunchKernelGGL((stream_only<K, 1, 1>), dim3(grid), dim3(256), 0, s, W, sh.N, out); }
    else if (rpw == 2) { if (NR == 2) hipLaunchKernelGGL((stream_only<K, 2, 2>), dim3(grid), dim3(256), 0, s, W, sh.N, out);
                         else hipLaunchKernelGGL((stream_only<K, 2, 1>), dim3(grid), dim3(256), 0, s, W, sh.N, out); }
    else { if (NR == 2) hipLaunchKernelGGL((stream_only<K, 4, 2>), dim3(grid), dim3(256), 0, s, W, sh.N, out);
           else hipLaunchKernelGGL((stream_only<K, 4, 1>), dim3(grid), dim3(256), 0, s, W, sh.N, out); }
}

static void one(const Bufs &b, const Shape &sh, const uint16_t *W, hipStream_t s) {
    if (b.variant == 0) {
        qasr::GemvArgs g{};
        g.W = W; g.K = sh.K; g.N = sh.N; g.M = 1; g.eps = 1e-6f;
        if (sh.norm) { g.x = b.x; g.ldx = sh.K; g.norm_w = b.nw; } else { g.xh = b.xh; g.ldxh = sh.K; }
        if (sh.swiglu) { g.out_f16 = b.out16; g.ldo16 = sh.N; qasr::launch_gemv(qasr::EPI_SWIGLU_F16, g, s); }
        else { g.out_f32 = b.out; g.ldo = sh.N; if (!sh.norm) { g.res = b.res; g.ldr = sh.N; } qasr::launch_gemv(qasr::EPI_F32, g, s); }
    } else if (b.variant == 1) {
        WArgs a{};
        a.x = b.x; a.xh = b.xh; a.norm_w = b.nw; a.W = W; a.res = sh.norm ? nullptr : b.res; a.out = b.out; a.out16 = b.out16;
        a.N = sh.N; a.eps = 1e-6f;
        switch (sh.K) {
            case 1024: launch_wave_k<1024>(sh, a, b.rpw, s); break;
            case 2048: launch_wave_k<2048>(sh, a, b.rpw, s); break;
            case 3072: launch_wave_k<3072>(sh, a, b.rpw, s); break;
        }
    } else if (b.variant == 2) {
        switch (sh.K) {
            case 1024: launch_stream_k<1024>(sh, W, b.out, b.rpw, s); break;
            case 2048: launch_stream_k<2048>(sh, W, b.out, b.rpw, s); break;
            case 3072: launch_stream_k<3072>(sh, W, b.out, b.rpw, s); break;
        }
    } else {
        const int grid = (sh.N + 4 * b.rpw - 1) / (4 * b.rpw);
        hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, s, b.out);
    }
}

static const Shape SH[4] = {{"qkv  4096x1024 +norm", 4096, 1024, true, false},
                            {"o    1024x2048 +res ", 1024, 2048, false, false},
                            {"gu   3072x1024 swiglu", 3072, 1024, true, true},
                            {"down 1024x3072 +res ", 1024, 3072, false, false}};
static std::vector<uint16_t *> g_w[4];
static Bufs *g_b;
static int g_shape;

static void body_shape(hipStream_t s, void *) {
    for (int l = 0; l < g_b->NL; l++) one(*g_b, SH[g_shape], g_w[g_shape][l], s);
}
static void body_layer(hipStream_t s, void *) {
    for (int l = 0; l < 28; l++)
        for (int k = 0; k < 4; k++) one(*g_b, SH[k], g_w[k][l], s);
}

int main() {
    const int NL = 64;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Bufs b{};
    b.NL = NL;
    CK(hipMalloc(&b.x, 16384 * 4)); CK(hipMalloc(&b.nw, 16384 * 4)); CK(hipMalloc(&b.res, 16384 * 4)); CK(hipMalloc(&b.out, 16384 * 4));
    CK(hipMalloc(&b.xh, 16384 * 2)); CK(hipMalloc(&b.out16, 16384 * 2));
    std::vector<float> hx(16384);
    for (int i = 0; i < 16384; i++) hx[i] = 0.01f * ((i * 37) % 101 - 50);
    CK(hipMemcpy(b.x, hx.data(), 16384 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b.nw, hx.data(), 16384 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b.res, hx.data(), 16384 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(b.xh, 0x3c, 16384 * 2));
    for (int k = 0; k < 4; k++) {
        const size_t n = (size_t)SH[k].N * (SH[k].swiglu ? 2 : 1) * SH[k].K;
        for (int l = 0; l < NL; l++) {
            uint16_t *w;
            CK(hipMalloc(&w, n * 2));
            CK(hipMemset(w, 0x11, n * 2));
            g_w[k].push_back(w);
        }
    }
    g_b = &b;
    const char *vn[4] = {"cur", "wave", "stream", "empty"};
    for (int k = 0; k < 4; k++) {
        g_shape = k;
        for (int v = 0; v < 4; v++)
            for (int rpw : {1, 2, 4}) {
                if (v == 0 && rpw > 1) continue;
                b.variant = v;
                b.rpw = rpw;
                const float us = time_graph(s, 10, body_shape, nullptr, NL);
                const double mb = (double)SH[k].N * (SH[k].swiglu ? 2 : 1) * SH[k].K * 2 / 1e6;
                printf("%-22s %-6s rpw %d: %7.2f us/launch  (%6.0f GB/s)\n", SH[k].name, vn[v], rpw, us, mb * 1e-3 / (us * 1e-6));
            }
    }
    for (int v = 0; v < 2; v++)
        for (int rpw : {1, 2, 4}) {
            if (v == 0 && rpw > 1) continue;
            b.variant = v;
            b.rpw = rpw;
            const float us = time_graph(s, 10, body_layer, nullptr, 28);
            printf("layer chain (qkv,o,gu,down) %-6s rpw %d: %7.2f us/layer\n", vn[v], rpw, us);
        }
    // correctness of wave vs cur on each shape (same math, same order)
    for (int k = 0; k < 4; k++) {
        std::vector<float> o0(SH[k].N), o1(SH[k].N);
        std::vector<uint16_t> h0(SH[k].N), h1(SH[k].N);
        b.rpw = 2;
        b.variant = 0; one(b, SH[k], g_w[k][0], s); CK(hipStreamSynchronize(s));
        CK(hipMemcpy(o0.data(), b.out, SH[k].N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h0.data(), b.out16, SH[k].N * 2, hipMemcpyDeviceToHost));
        b.variant = 1; one(b, SH[k], g_w[k][0], s); CK(hipStreamSynchronize(s));
        CK(hipMemcpy(o1.data(), b.out, SH[k].N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h1.data(), b.out16, SH[k].N * 2, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < SH[k].N; i++) bad += SH[k].swiglu ? (h0[i] != h1[i]) : (o0[i] != o1[i]);
        printf("%s: wave vs cur mismatches %d / %d\n", SH[k].name, bad, SH[k].N);
    }
    return 0;
}
