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
__device__ __forceinline__ void ld_sc1_x4_6(const uint16_t *p, u32x4 *v) {
    asm volatile(
        "global_load_dwordx4 %0, %6, off sc1\n\t"
        "global_load_dwordx4 %1, %6, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %6, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %6, off offset:3072 sc1\n\t"
        "global_load_dwordx4 %4, %7, off sc1\n\t"
        "global_load_dwordx4 %5, %7, off offset:1024 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5])
        : "v"(p), "v"(p + 2048)
        : "memory");
}

struct FfnCtl {
    unsigned int *cnt, *cnt_next;   // this layer's 32 arrival shards (16-word stride), the next layer's
    unsigned int *err;              // sticky device error word
    int wdelay, delay, poll_limit, fence;
};

template <int K, int F>
__global__ __launch_bounds__(256) void ffn1_kernel(GemvArgs g, GemvArgs d, FfnCtl c) {
    constexpr int NT = K / 512, NTD = F / 512, NGU = F / 4;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    stamp_start(g.stamp);
    if (blockIdx.x >= NGU) {   // ---- down projection
        const int j = blockIdx.x - NGU, row = j * 4 + wid;
        if (d.trace && threadIdx.x == 0) d.trace[j * 8] = rt_now();
        for (int i = 0; i < c.wdelay; i++) __builtin_amdgcn_s_sleep(8);   // let the gate/up stream go first
        half8 wv[NTD];
#pragma unroll
        for (int t = 0; t < NTD; t++) wv[t] = __builtin_nontemporal_load((const half8 *)(d.W + (long)row * F + t * 512 + lane * 8));
        // one polling lane per block, and only once the gate/up stream is
        // nearly done: pollers beside a weight stream cost it bandwidth
        // (MI355X_MICROARCH.md, polling-cost)
        __shared__ int ready;
        if (wid == 0) {   // lane s polls shard s; every shard holds NGU / 32 arrivals when done
            for (int i = 0; i < c.delay; i++) __builtin_amdgcn_s_sleep(8);
            int ok = 0;
            for (int it = 0; it < c.poll_limit; it++) {
                const unsigned v = lane < 32 ? __hip_atomic_load(c.cnt + lane * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
                if (__all(v >= (unsigned)(NGU / 32))) { ok = 1; break; }
                __builtin_amdgcn_s_sleep(8);
            }
            if (c.fence) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (lane == 0) {
                ready = ok;
                if (!ok) __hip_atomic_fetch_or(c.err, (unsigned)DEVERR_FFN_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (!ready) { stamp_end(g.stamp); return; }   // reported through the error word; x keeps its old row
        u32x4 xv[NTD];
        static_assert(NTD == 6, "ld_sc1_x4_6 covers F = 3072");
        ld_sc1_x4_6(d.xh + lane * 8, xv);
        const float res = d.res[row];
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < NTD; t++) {
            const half8 h = __builtin_bit_cast(half8, xv[t]);
#pragma unroll
            for (int e = 0; e < 8; e++) acc = fmaf((float)wv[t][e], (float)h[e], acc);
        }
        acc = wave_sum(acc);
        if (lane == 0) d.out_f32[row] = fadd_rn(acc, res);
        if (d.trace && threadIdx.x == 0) d.trace[j * 8 + 1] = rt_now();
        stamp_end(g.stamp);
        return;
    }
    // ---- gate/up (16-row interleave: output o = rows 32 (o / 16) + o % 16 and + 16)
    if (g.trace && threadIdx.x == 0) g.trace[blockIdx.x * 8] = rt_now();
    if (blockIdx.x == 0 && threadIdx.x < 32) {   // re-arm: the next layer's shards and the fused o-proj's counters
        c.cnt_next[threadIdx.x * 16] = 0u;
        if (d.zero8 && threadIdx.x < 8) d.zero8[threadIdx.x * 16] = 0u;
    }
    const int o = blockIdx.x * 4 + wid;
    half8 wv[2][NT];
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
        for (int t = 0; t < NT; t++)
            wv[q][t] = __builtin_nontemporal_load((const half8 *)(g.W + (32L * (o >> 4) + (o & 15) + 16 * q) * K + t * 512 + lane * 8));
    float xf[NT][8];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const float4 a = *(const float4 *)(g.x + t * 512 + lane * 8);
        const float4 b = *(const float4 *)(g.x + t * 512 + lane * 8 + 4);
        xf[t][0] = a.x; xf[t][1] = a.y; xf[t][2] = a.z; xf[t][3] = a.w;
        xf[t][4] = b.x; xf[t][5] = b.y; xf[t][6] = b.z; xf[t][7] = b.w;
    }
    double ss = 0.0;   // ggml_rms_norm: double sum of fp32 squares
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int e = 0; e < 8; e++) ss += (double)(xf[t][e] * xf[t][e]);
    ss = wave_sum_d(ss);
    const float scale = 1.0f / sqrtf((float)(ss / K) + g.eps);
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const float4 a = *(const float4 *)(g.norm_w + t * 512 + lane * 8);
        const float4 b = *(const float4 *)(g.norm_w + t * 512 + lane * 8 + 4);
        const float w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; e++) xf[t][e] = (float)f2h(fmul_rn(fmul_rn(xf[t][e], scale), w[e]));
    }
    float acc[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        acc[q] = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int e = 0; e < 8; e++) acc[q] = fmaf((float)wv[q][t][e], xf[t][e], acc[q]);
        acc[q] = wave_sum(acc[q]);
    }
    __shared__ uint16_t outs[4];
    if (lane == 0) outs[wid] = f_to_u16(silu1(acc[0]) * acc[1]);
    __syncthreads();
    if (wid == 0) {
        if (lane < 2)
            __hip_atomic_store((uint32_t *)(g.out_f16 + blockIdx.x * 4) + lane, (uint32_t)outs[2 * lane] | ((uint32_t)outs[2 * lane + 1] << 16),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (c.fence) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) __hip_atomic_fetch_add(c.cnt + (blockIdx.x & 31) * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (g.trace && threadIdx.x == 0) g.trace[blockIdx.x * 8 + 1] = rt_now();
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
