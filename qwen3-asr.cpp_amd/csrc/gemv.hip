// gemv.hip -- batch-1 decode projections, one wave per output row group.
//
// The decode step at B = 1 is a chain of small weight-streaming launches
// (4-13 MB each), so a launch's fixed cost -- not its bandwidth -- sets the
// time.  This kernel has no LDS and no workgroup barrier: every wave loads
// its RPW weight rows (16-byte non-temporal loads, all issued first), then its
// own slice of x straight from L2 (each lane multiplies x[t*512 + 8*lane ..+8]
// with the same slice of every row), redoes the RMS norm for itself (one
// wave-wide double sum instead of a block reduction), and writes its outputs
// from lane 0.  Per-lane products and the wave_sum order are those of
// gemm.hip's gemv_kernel, so the two are bit-identical (tools/gemv_floor.hip
// measures both: 16.9 -> 13.9 us per decoder layer's four projections).
//
// Numerics = ggml_mul_mat with F16 weights (SURVEY.md §8(a) i): x rounded to
// fp16 (after rms_norm * w, text_decoder.cpp:480-481/546-547), fp32 sums.
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

__device__ __forceinline__ float silu1(float g) { return g / (1.0f + expf(-g)); }

template <int EPI, int K, int RPW>
__global__ __launch_bounds__(256) void gemv1_kernel(GemvArgs g) {
    constexpr int NT = (K + 511) / 512;
    constexpr bool PART = K % 512 != 0;   // lanes past K hold x = 0 (clamped weight loads)
    constexpr int NR = EPI == EPI_SWIGLU_F16 ? 2 : 1;   // gate/up rows per output (16-row interleave)
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    trace_mark(g.trace, 0);
    if (g.zero8 && blockIdx.x == 0 && threadIdx.x < 8) g.zero8[threadIdx.x * 16] = 0u;   // fused o-proj counters
    half8 wv[RPW][NR][NT];
#pragma unroll
    for (int r = 0; r < RPW; r++)
#pragma unroll
        for (int q = 0; q < NR; q++)
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const int o = min(row0 + r, g.N - 1);
                const long wrow = NR == 2 ? 32L * (o >> 4) + (o & 15) + 16 * q : o;
                wv[r][q][t] = __builtin_nontemporal_load((const half8 *)(g.W + wrow * K + min(t * 512 + lane * 8, K - 8)));
            }
    float xf[NT][8];
    if (g.xh) {
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const half8 h = *(const half8 *)(g.xh + min(t * 512 + lane * 8, K - 8));
#pragma unroll
            for (int e = 0; e < 8; e++) xf[t][e] = (float)h[e];
        }
        if (PART && lane * 8 >= K - (NT - 1) * 512)
#pragma unroll
            for (int e = 0; e < 8; e++) xf[NT - 1][e] = 0.f;
    } else {
        if (g.embd_ids) {   // decode layer 0: x = token_embd[id] (fp16 -> fp32)
            const uint16_t *er = g.embd + (long)g.embd_ids[0] * K;
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const half8 h = *(const half8 *)(er + min(t * 512 + lane * 8, K - 8));
#pragma unroll
                for (int e = 0; e < 8; e++) xf[t][e] = (float)h[e];
            }
            if (g.x_store && blockIdx.x == 0 && threadIdx.x < 64)   // residual stream for the later layers
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    if (t * 512 + lane * 8 >= K) continue;
                    *(float4 *)(g.x_store + t * 512 + lane * 8) = make_float4(xf[t][0], xf[t][1], xf[t][2], xf[t][3]);
                    *(float4 *)(g.x_store + t * 512 + lane * 8 + 4) = make_float4(xf[t][4], xf[t][5], xf[t][6], xf[t][7]);
                }
        } else {
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const int k = min(t * 512 + lane * 8, K - 8);
                const float4 a = *(const float4 *)(g.x + k);
                const float4 b = *(const float4 *)(g.x + k + 4);
                xf[t][0] = a.x; xf[t][1] = a.y; xf[t][2] = a.z; xf[t][3] = a.w;
                xf[t][4] = b.x; xf[t][5] = b.y; xf[t][6] = b.z; xf[t][7] = b.w;
            }
        }
        if (PART && lane * 8 >= K - (NT - 1) * 512)
#pragma unroll
            for (int e = 0; e < 8; e++) xf[NT - 1][e] = 0.f;
        float scale = 1.0f;
        if (g.norm_w) {   // ggml_rms_norm: double sum of fp32 squares
            double ss = 0.0;
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int e = 0; e < 8; e++) ss += (double)(xf[t][e] * xf[t][e]);
            ss = wave_sum_d(ss);
            scale = 1.0f / sqrtf((float)(ss / K) + g.eps);
        }
#pragma unroll
        for (int t = 0; t < NT; t++) {
            float w[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
            if (g.norm_w) {
                const int k = min(t * 512 + lane * 8, K - 8);
                const float4 a = *(const float4 *)(g.norm_w + k);
                const float4 b = *(const float4 *)(g.norm_w + k + 4);
                w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                float v = xf[t][e];
                if (g.norm_w) v = fmul_rn(fmul_rn(v, scale), w[e]);
                xf[t][e] = (float)f2h(v);
            }
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
        if (lane == 0 && o < g.N) {
            if constexpr (EPI == EPI_SWIGLU_F16) {
                g.out_f16[o] = f_to_u16(silu1(acc[0]) * acc[1]);
            } else {
                float y = acc[0];
                if (g.bias) y = fadd_rn(y, g.bias[o]);
                if constexpr (EPI == EPI_F16) {
                    g.out_f16[o] = f_to_u16(y);
                } else {
                    if (g.res) y = fadd_rn(y, g.res[o]);
                    g.out_f32[o] = y;
                }
            }
        }
    }
    if (g.trace) { __syncthreads(); trace_mark(g.trace, 1); }
}

template <int EPI, int K, int RPW>
static void run_gemv1(const GemvArgs &g, hipStream_t s) {
    const int grid = (g.N + 4 * RPW - 1) / (4 * RPW);
    hipLaunchKernelGGL((gemv1_kernel<EPI, K, RPW>), dim3(grid), dim3(256), 0, s, g);
}

template <int EPI, int K>
static void gemv1_rpw(const GemvArgs &g, hipStream_t s) {
    // 2 rows per wave only for the wide QKV projection (tools/gemv_floor.hip)
    if (EPI != EPI_SWIGLU_F16 && g.N >= 4096) run_gemv1<EPI, K, 2>(g, s);
    else run_gemv1<EPI, K, 1>(g, s);
}

template <int EPI>
static bool gemv1_k(const GemvArgs &g, hipStream_t s) {
    switch (g.K) {
        case 256: gemv1_rpw<EPI, 256>(g, s); return true;
        case 512: gemv1_rpw<EPI, 512>(g, s); return true;
        case 1024: gemv1_rpw<EPI, 1024>(g, s); return true;
        case 2048: gemv1_rpw<EPI, 2048>(g, s); return true;
        case 3072: gemv1_rpw<EPI, 3072>(g, s); return true;
        default: return false;
    }
}

// single-row f16 projections of the decode step; false = not covered (the
// caller falls back to gemm.hip's multi-row kernel)
bool launch_gemv1(int epi, const GemvArgs &g, hipStream_t s) {
    if (g.M != 1 || g.Wd) return false;
    switch (epi) {
        case EPI_F32: return gemv1_k<EPI_F32>(g, s);
        case EPI_F16: return gemv1_k<EPI_F16>(g, s);
        case EPI_SWIGLU_F16: return gemv1_k<EPI_SWIGLU_F16>(g, s);
        default: return false;
    }
}

}  // namespace qasr
