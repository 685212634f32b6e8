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
#include "ffn_roles.h"

namespace qasr {

template <int EPI, int K, int RPW>
__global__ __launch_bounds__(256) void gemv1_kernel(GemvArgs g) {
    constexpr int NT = (K + 511) / 512;
    constexpr bool PART = K % 512 != 0;   // lanes past K hold x = 0 (clamped weight loads)
    constexpr int NR = EPI == EPI_SWIGLU_F16 ? 2 : 1;   // gate/up rows per output (16-row interleave)
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    trace_mark(g.trace, 0);
    stamp_start(g.stamp);
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
    stamp_end(g.stamp);
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

// ------------------------------------------------ batch 1: gate/up + down
// One launch for the batch-1 FFN (text_decoder.cpp:545-560: rms_norm * w ->
// silu(gate) * up -> down + residual).  Blocks [0, F/4): the gate/up GEMV
// (gemv1_kernel<EPI_SWIGLU_F16, K, 1> arithmetic, 4 outputs per block); the
// block's 4 fp16 outputs leave as two write-through 32-bit stores, the wave
// drains, and its lane 0 counts the block into shard b % 32 of the layer's
// counter (MI355X_MICROARCH.md inter-workgroup hand-off, row 2 with sharded
// replicas: one counter of 768 arrivals serialises ~12 ns per atomic at the
// memory side, ~9 us; 32 shards hold 24 each).  Blocks past F/4: the down
// projection (gemv1_kernel<EPI_F32, F, 1> arithmetic + residual), which
// requests its weights once the gate/up stream is under way (both at once
// just split the same HBM queue: measured slower than two launches), then
// polls the 32 shards (one lane each, one wave) and reads the activation
// with sc1 loads -- the down weight stream overlaps the gate/up one instead of
// following a kernel boundary.  Counters are per layer; block 0 re-arms the
// next layer's (its last use ended a whole step ago), so the fusion needs two
// or more layers.  The residual x is read by the gate/up blocks and rewritten
// (row by row) by the down blocks only after every gate/up block has arrived.
template <int K, int F>
__global__ __launch_bounds__(256) void ffn1_kernel(GemvArgs g, GemvArgs d, FfnCtl c) {
    constexpr int NGU = F / 4;
    stamp_start(g.stamp);
    if (blockIdx.x >= NGU) ffn_dn_role<F, 1>(d, c, blockIdx.x - NGU, NGU / 32);
    else ffn_gu_role<K, 1>(g, d, c, blockIdx.x);
    stamp_end(g.stamp);
}

// the plain batch-1 f16 FFN (K = 1024, F = 3072) in one launch when every
// block is co-resident; false = not covered (two launch_gemv calls instead)
bool launch_ffn1(const GemvArgs &g, const GemvArgs &d, unsigned int *cnt, unsigned int *cnt_next, const FuseCfg &cfg,
                 hipStream_t s, bool dry) {
    if (!cfg.ffn || !cfg.err || !cnt || !cnt_next || cnt_next == cnt || g.M != 1 || d.M != 1 || g.Wd || d.Wd || g.K != 1024 ||
        g.N != 3072 || !g.x || g.xh || !g.norm_w || g.embd_ids || !g.out_f16 || d.K != 3072 || d.N != 1024 || d.xh != g.out_f16 ||
        !d.res || d.bias || d.norm_w || !d.out_f32)
        return false;
    const int grid = 3072 / 4 + 1024 / 4;
    if (grid > cfg.slots_ffn) return false;   // down blocks wait on gate/up blocks: all must be resident
    if (dry) return true;
    // delays in s_sleep(8) units (~0.2 us): down weights requested ~3 us after the
    // gate/up ones, first poll ~1 us later (round-1 delay sweep, 92 s decode:
    // unfused 224.8 ms; 12/4 217.9, 14/4 208.2 (x3), 16/4 210.0, 14/2 210.8, 14/6 210.0, 20/6 221.0)
    const FfnCtl c{cnt, cnt_next, cfg.err, cfg.ffn_wdelay, cfg.ffn_delay, cfg.poll_limit, cfg.fence};
    hipLaunchKernelGGL((ffn1_kernel<1024, 3072>), dim3(grid), dim3(256), 0, s, g, d, c);
    return true;
}

static int slots_of(const void *kernel) {
    int nb = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0) != hipSuccess)
        return 0;   // unknown capacity: never fuse
    return nb * cus;
}

int fused_slots_ffn() { return slots_of(reinterpret_cast<const void *>(ffn1_kernel<1024, 3072>)); }

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
