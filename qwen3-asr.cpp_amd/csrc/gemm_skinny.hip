// gemm_skinny.hip -- weight-streaming MFMA GEMM for decode batches
// (9 <= M <= 128 rows: the batched decode step's projections and LM head).
//
// The tiled GEMM (gemm.hip) gives a 64-row batch only N/64 workgroups -- 64
// for the 4096-wide QKV projection -- so a batch-64 decode step ran its
// weight streams on a quarter of the CUs (32 us for 8 MB).  Here a workgroup
// owns only 16*NT output columns and its KW waves split K, so the grid is
// N/(16 NT) workgroups of up to 1024 waves in all; every weight byte is read
// once (nontemporal), the activations (<= 64 x K fp16) come from L2.
//
// Weights go straight from global memory into MFMA fragments: per 128-wide
// K chunk and sub-step s, lane (q = lane>>4, c = lane&15) loads k = 32s + 8q
// .. +8 of row c, so one load instruction covers 64 contiguous bytes of each
// of 16 rows (the natural v_mfma_f32_16x16x32_f16 layout; fp16 x fp16
// products summed in fp32 = ggml_mul_mat F16 numerics, gemm.hip header).
// The activations (re-read from L2 by every column tile) go through LDS by
// LDS-DMA in whole 256-B row segments (one wave's K chunk, XOR-swizzled 16-B
// chunks so the fragment reads of 16 rows hit distinct banks).
// The KW per-wave partial tiles are summed through LDS in wave order
// (deterministic), then the epilogue runs the same per-element code as the
// tiled GEMM: +bias, +residual, fp16 / SwiGLU / argmax outputs.
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

__device__ __forceinline__ float silu_s(float g) { return g / (1.0f + expf(-g)); }
// an s_waitcnt vmcnt immediate: 63 at most (a smaller count only waits longer)
constexpr int vmc(int x) { return x > 63 ? 63 : x; }

// Residual prefetch: epilogue element e -> (tile, row in tile, column in
// tile); the residual values a thread adds are requested at kernel entry, so
// their latency hides under the K loop.
template <int MT, int NT, int KW, int EPI>
struct SkinnyEpi {
    static constexpr int NTILE = MT * NT;
    static constexpr int EPT = (NTILE * 256 + 64 * KW - 1) / (64 * KW);
    float resv[EPT];

    __device__ __forceinline__ void prefetch(const GemmArgs &g, int m0, int n0, int tid) {
        if constexpr (EPI == EPI_F32) {
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const int e = tid + k * 64 * KW;
                const int t = e >> 8, rin = (e >> 4) & 15, cin = e & 15;
                const int i = t / NT, j = t - i * NT;
                const int row = m0 + i * 16 + rin, col = n0 + j * 16 + cin;
                resv[k] = (e < NTILE * 256 && row < g.M && g.res) ? g.res[(long)row * g.ldr + col] : 0.f;
            }
        }
    }

    // red: the KW waves' partial tiles in the MFMA C layout ((row, col) in lane
    // ((row >> 2) << 4) | col, register row & 3), summed here in wave order
    __device__ __forceinline__ void run(const GemmArgs &g, floatx4 (*red)[NTILE][64], unsigned long long *rmax, int m0,
                                        int n0, int tid) {
        const int M = g.M;
        auto tile_val = [&](int t, int rin, int cin) {
            const int l = ((rin >> 2) << 4) | cin, r = rin & 3;
            float v = red[0][t][l][r];
#pragma unroll
            for (int w = 1; w < KW; w++) v += red[w][t][l][r];
            return v;
        };
        if constexpr (EPI == EPI_SWIGLU_Q8) {
            // silu(g) * u of the block's NT / 2 * 16 output columns (whole Q8_0
            // blocks: NT % 4 == 0) through LDS, then quantize_q8_rows_kernel's
            // arithmetic per 32-block: 8 lanes of 4 values, amax by xor shuffles
            static_assert(NT % 4 == 0, "whole 32-column blocks (and MT * NT * 32 lane groups: whole waves)");
            constexpr int OC = NT / 2 * 16;
            __shared__ __attribute__((aligned(16))) float vq[MT * 16][OC];
            for (int e = tid; e < MT * (NT / 2) * 256; e += 64 * KW) {
                const int tp = e >> 8, rin = (e >> 4) & 15, cin = e & 15;
                const int i = tp / (NT / 2), p = tp - i * (NT / 2);
                const float gt = tile_val(i * NT + 2 * p, rin, cin), up = tile_val(i * NT + 2 * p + 1, rin, cin);
                vq[i * 16 + rin][p * 16 + cin] = silu_s(gt) * up;
            }
            __syncthreads();
            for (int u = tid; u < MT * 16 * OC / 4; u += 64 * KW) {   // wave-uniform trip count
                const int rl = u / (OC / 4), c4 = u - rl * (OC / 4), row = m0 + rl;
                const float4 v = *(const float4 *)&vq[rl][4 * c4];
                float am = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
                am = fmaxf(am, __shfl_xor(am, 1, 64));
                am = fmaxf(am, __shfl_xor(am, 2, 64));
                am = fmaxf(am, __shfl_xor(am, 4, 64));
                if (row >= M) continue;
                const int col = n0 / 2 + 4 * c4;
                *(uint32_t *)(g.out_q + (long)row * g.ldoq + col) =
                    (uint32_t)(uint8_t)q8_quant(v.x, am) | (uint32_t)(uint8_t)q8_quant(v.y, am) << 8 |
                    (uint32_t)(uint8_t)q8_quant(v.z, am) << 16 | (uint32_t)(uint8_t)q8_quant(v.w, am) << 24;
                if ((c4 & 7) == 0) g.out_d[(long)row * (g.ldoq / 32) + col / 32] = q8_scale(am);
            }
        } else if constexpr (EPI == EPI_SWIGLU_F16 || EPI == EPI_SWIGLU_F32) {
            // interleaved 16-row [gate | up] weight blocks: tiles 2p / 2p+1
            for (int e = tid; e < MT * (NT / 2) * 256; e += 64 * KW) {
                const int tp = e >> 8, rin = (e >> 4) & 15, cin = e & 15;
                const int i = tp / (NT / 2), p = tp - i * (NT / 2);
                const int row = m0 + i * 16 + rin;
                if (row >= M) continue;
                const float gt = tile_val(i * NT + 2 * p, rin, cin), up = tile_val(i * NT + 2 * p + 1, rin, cin);
                const float v = silu_s(gt) * up;
                const int ocol = n0 / 2 + p * 16 + cin;
                if constexpr (EPI == EPI_SWIGLU_F32) g.out_f32[(long)row * g.ldo + ocol] = v;
                else g.out_f16[(long)row * g.ldo16 + ocol] = f_to_u16(v);
            }
        } else {
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const int e = tid + k * 64 * KW;
                if (e >= NTILE * 256) break;
                const int t = e >> 8, rin = (e >> 4) & 15, cin = e & 15;
                const int i = t / NT, j = t - i * NT;
                const int rl = i * 16 + rin, row = m0 + rl;
                const int col = n0 + j * 16 + cin;
                float v = tile_val(t, rin, cin);
                if (row >= M) continue;
                if constexpr (EPI == EPI_ARGMAX) {
                    if (g.out_f32) g.out_f32[(long)row * g.ldo + col] = v;
                    if (g.n_valid == 0 || col < g.n_valid) atomicMax(&rmax[rl], argmax_key(v, col));
                } else {
                    if (g.bias) v = fadd_rn(v, g.bias[col]);
                    if constexpr (EPI == EPI_F16) {
                        g.out_f16[(long)row * g.ldo16 + col] = f_to_u16(v);
                    } else {
                        if (g.res) v = fadd_rn(v, resv[k]);
                        g.out_f32[(long)row * g.ldo + col] = v;
                    }
                }
            }
            if constexpr (EPI == EPI_ARGMAX) {
                __syncthreads();
                if (tid < MT * 16 && m0 + tid < M) atomicMax(g.amax + m0 + tid, rmax[tid]);
            }
        }
    }
};

typedef __attribute__((address_space(3))) void lds_void_s;
typedef __attribute__((address_space(1))) void glb_void_s;
__device__ __attribute__((aligned(64))) uint32_t g_zero_line_s[16];

// VAR: diagnostic knob for tools/skinny_bench.hip (1 = no activation loads,
// 2 = no weight loads, 4 = activations through LDS by LDS-DMA, 8 = weights with
// the default cache policy instead of nontemporal loads); the engine launches 4
// and 4 | 8 (GemmArgs::wdef)
// CPW > 0 (with VAR 4): every one of the wave's CPW K chunks (nch == KW * CPW)
// requested at entry -- LDS-DMA pieces and weight fragments, each chunk in an
// LDS region of its own -- then consumed in the same order: the same fragments
// and accumulation order as the one-chunk-at-a-time loop (bit-identical), but
// one memory latency per launch instead of one per chunk (the batch decode's
// o / down / gate-up projections waited 2-3 HBM latencies a launch)
template <int MT, int NT, int KW, int EPI, int VAR = 0, int CPW = 0>
__global__ __launch_bounds__(64 * KW) void gemm_skinny_kernel(GemmArgs g) {
    constexpr int NTILE = MT * NT;
    constexpr bool ALDS = (VAR & 4) != 0;
    // VAR 4: one K chunk (MT*16 rows x 128 halves, 16-B chunks XOR-swizzled by
    // row) per wave (CPW of them with CPW > 0), in the same LDS as the
    // partial-tile reduction after the loop
    constexpr int RED_B = KW * NTILE * 64 * 16, ALDS_B = ALDS ? KW * MT * 16 * 128 * 2 * (CPW > 0 ? CPW : 1) : 0;
    static_assert((RED_B > ALDS_B ? RED_B : ALDS_B) + 512 <= 160 * 1024, "LDS per workgroup");
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[RED_B > ALDS_B ? RED_B : ALDS_B];
    floatx4 (*red)[NTILE][64] = reinterpret_cast<floatx4 (*)[NTILE][64]>(lds_raw);
    uint16_t *alds = reinterpret_cast<uint16_t *>(lds_raw);
    __shared__ unsigned long long rmax[64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n0 = blockIdx.x * 16 * NT, m0 = blockIdx.y * 16 * MT;
    const int M = g.M;
    const int q = lane >> 4, c16 = lane & 15;

    const u32x4 *wrow[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) wrow[t] = (const u32x4 *)(g.W + (long)(n0 + t * 16 + c16) * g.ldw + q * 8);
    const u32x4 *arow[MT];
    bool aok[MT];
#pragma unroll
    for (int t = 0; t < MT; t++) {
        const int m = m0 + t * 16 + c16;
        aok[t] = m < M;
        arow[t] = (const u32x4 *)(g.A + (long)(aok[t] ? m : 0) * g.lda + q * 8);
    }
    SkinnyEpi<MT, NT, KW, EPI> epi;
    epi.prefetch(g, m0, n0, tid);

    floatx4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NT; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int nch = g.K >> 7;
    u32x4 wb[2][NT][4], ab[2][MT][4];
    auto load = [&](int buf, int c) {
        const int off = c * 16;   // 128 halves = 16 u32x4
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int s = 0; s < 4; s++)
                wb[buf][t][s] = (VAR & 2) ? u32x4{1u, 2u, 3u, (unsigned)c} : (VAR & 8) ? wrow[t][off + 4 * s] : __builtin_nontemporal_load(wrow[t] + off + 4 * s);
#pragma unroll
        for (int t = 0; t < MT; t++)
#pragma unroll
            for (int s = 0; s < 4; s++)
                ab[buf][t][s] = (VAR & 1) ? u32x4{4u, 5u, 6u, (unsigned)c} : aok[t] ? arow[t][off + 4 * s] : u32x4{0u, 0u, 0u, 0u};
    };
    auto mma = [&](int buf) {
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int i = 0; i < MT; i++)
#pragma unroll
                for (int j = 0; j < NT; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, ab[buf][i][s]),
                                                                       __builtin_bit_cast(half8, wb[buf][j][s]), acc[i][j], 0, 0, 0);
    };
    if constexpr (ALDS && CPW > 0) {
        static_assert(CPW <= 4, "the per-chunk vmcnt waits below are written out for at most 4 chunks");
        uint16_t *my = alds + wid * (CPW * MT * 16 * 128);
        u32x4 wq[CPW][NT][4];
#pragma unroll
        for (int k = 0; k < CPW; k++) {
            const int c = wid + k * KW;
#pragma unroll
            for (int p = 0; p < MT * 4; p++) {   // 1 KiB = 4 rows of 256 B per piece
                const int r = p * 4 + (lane >> 4), ch = (lane & 15) ^ (r & 15);
                const int m = m0 + r;
                const uint16_t *src = m < M ? g.A + (long)m * g.lda + c * 128 + ch * 8 : (const uint16_t *)g_zero_line_s;
                __builtin_amdgcn_global_load_lds((glb_void_s *)src, (lds_void_s *)(my + k * (MT * 16 * 128) + p * 512), 16, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++) wq[k][t][s4] = (VAR & 8) ? wrow[t][c * 16 + 4 * s4] : __builtin_nontemporal_load(wrow[t] + c * 16 + 4 * s4);
            asm volatile("" ::: "memory");   // chunk k's requests stay together, in chunk order (the waits below count them)
        }
#pragma unroll
        for (int k = 0; k < CPW; k++) {
            // chunk k's pieces and fragments landed: (MT + NT) * 4 loads per chunk, issued in chunk order
            // (vmcnt holds 63 at most: a smaller count only waits longer)
            if (k == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW - 1) * (MT + NT) * 4)) : "memory");
            else if (k == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW > 1 ? CPW - 2 : 0) * (MT + NT) * 4)) : "memory");
            else if (k == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW > 2 ? CPW - 3 : 0) * (MT + NT) * 4)) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW > 3 ? CPW - 4 : 0) * (MT + NT) * 4)) : "memory");
            const uint16_t *mk = my + k * (MT * 16 * 128);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int i = 0; i < MT; i++) {
                    const int r = i * 16 + c16, ch = (4 * s4 + q) ^ (r & 15);
                    const half8 a8 = *(const half8 *)(mk + r * 128 + ch * 8);
#pragma unroll
                    for (int j = 0; j < NT; j++)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, __builtin_bit_cast(half8, wq[k][j][s4]), acc[i][j], 0, 0, 0);
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if constexpr (ALDS) {
        uint16_t *my = alds + wid * (MT * 16 * 128);
        for (int c = wid; c < nch; c += KW) {
#pragma unroll
            for (int p = 0; p < MT * 4; p++) {   // 1 KiB = 4 rows of 256 B per piece
                const int r = p * 4 + (lane >> 4), ch = (lane & 15) ^ (r & 15);
                const int m = m0 + r;
                const uint16_t *src = m < M ? g.A + (long)m * g.lda + c * 128 + ch * 8 : (const uint16_t *)g_zero_line_s;
                __builtin_amdgcn_global_load_lds((glb_void_s *)src, (lds_void_s *)(my + p * 512), 16, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++) wb[0][t][s4] = (VAR & 8) ? wrow[t][c * 16 + 4 * s4] : __builtin_nontemporal_load(wrow[t] + c * 16 + 4 * s4);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int i = 0; i < MT; i++) {
                    const int r = i * 16 + c16, ch = (4 * s4 + q) ^ (r & 15);
                    const half8 a8 = *(const half8 *)(my + r * 128 + ch * 8);
#pragma unroll
                    for (int j = 0; j < NT; j++)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, __builtin_bit_cast(half8, wb[0][j][s4]), acc[i][j], 0, 0, 0);
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this chunk's reads done before the next pieces land
        }
    } else {
        int c = wid;
        if (c < nch) load(0, c);
        for (; c < nch; c += 2 * KW) {
            if (c + KW < nch) load(1, c + KW);
            mma(0);
            if (c + KW >= nch) break;
            if (c + 2 * KW < nch) load(0, c + 2 * KW);
            mma(1);
        }
    }

    if constexpr (ALDS) __syncthreads();   // every wave's chunk reads done before the reduction reuses the LDS
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NT; j++) red[wid][i * NT + j][lane] = acc[i][j];
    if constexpr (EPI == EPI_ARGMAX)
        if (tid < 64) rmax[tid] = 0ull;
    __syncthreads();
    epi.run(g, red, rmax, m0, n0, tid);
}

// ---------------------------------------------------------------- Q8_0
// ggml_mul_mat(W Q8_0, X): activations already quantised to int8 + fp32
// block scales (quantize_q8_kernel / the fused producers), weights int8 +
// fp16 block scales.  Per 32-wide block one v_mfma_i32_16x16x32_i8 from a
// zero accumulator gives the exact integer dot, then acc += (d_w * d_x) *
// sumi in fp32 -- the numerics of gemm_q8_kernel (gemm.hip).  Operands are
// 8-byte fragment loads (one instruction = 32 contiguous bytes of 16 rows).
template <int MT, int NT, int KW, int EPI, int VAR = 0, int CPW = 0>
__global__ __launch_bounds__(64 * KW) void gemm_skinny_q8_kernel(GemmArgs g) {
    constexpr int NTILE = MT * NT;
    constexpr bool ALDS = (VAR & 4) != 0;   // int8 activations through LDS-DMA, as gemm_skinny_kernel
    constexpr int RED_B = KW * NTILE * 64 * 16, ALDS_B = ALDS ? KW * MT * 16 * 128 * (CPW > 0 ? CPW : 1) : 0;
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[RED_B > ALDS_B ? RED_B : ALDS_B];
    floatx4 (*red)[NTILE][64] = reinterpret_cast<floatx4 (*)[NTILE][64]>(lds_raw);
    __shared__ unsigned long long rmax[64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n0 = blockIdx.x * 16 * NT, m0 = blockIdx.y * 16 * MT;
    const int M = g.M, nbk = g.K >> 5;
    const int q = lane >> 4, c16 = lane & 15;

    const int8_t *wrow[NT];
    const uint16_t *wdrow[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        wrow[t] = g.Wq + (long)(n0 + t * 16 + c16) * g.ldw + q * 8;
        wdrow[t] = g.Wd + (long)(n0 + t * 16 + c16) * nbk;
    }
    const int8_t *arow[MT];
    bool aok[MT];
    const float *adrow[MT][4];   // scales of the C-layout rows 4q + r of tile t
#pragma unroll
    for (int t = 0; t < MT; t++) {
        const int m = m0 + t * 16 + c16;
        aok[t] = m < M;
        arow[t] = g.Aq + (long)(aok[t] ? m : 0) * g.lda + q * 8;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int mr = m0 + t * 16 + 4 * q + r;
            adrow[t][r] = g.Ad + (long)(mr < M ? mr : 0) * g.ldad;
        }
    }
    SkinnyEpi<MT, NT, KW, EPI> epi;
    epi.prefetch(g, m0, n0, tid);

    floatx4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NT; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // one 128-wide K chunk = 4 blocks
    const int nch = g.K >> 7;
    long wb[2][NT][4], ab[2][MT][4];
    uint2 wd[2][NT];          // 4 fp16 weight scales of the chunk
    float4 ad[2][MT][4];      // [tile][r] 4 activation block scales of the chunk
    auto load = [&](int buf, int c) {
#pragma unroll
        for (int t = 0; t < NT; t++) {
#pragma unroll
            for (int u = 0; u < 4; u++) wb[buf][t][u] = __builtin_nontemporal_load((const long *)(wrow[t] + c * 128 + u * 32));
            wd[buf][t] = *(const uint2 *)(wdrow[t] + c * 4);
        }
#pragma unroll
        for (int t = 0; t < MT; t++) {
#pragma unroll
            for (int u = 0; u < 4; u++) ab[buf][t][u] = aok[t] ? *(const long *)(arow[t] + c * 128 + u * 32) : 0l;
#pragma unroll
            for (int r = 0; r < 4; r++) ad[buf][t][r] = *(const float4 *)(adrow[t][r] + c * 4);
        }
    };
    auto mma = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            float sb[NT];
#pragma unroll
            for (int j = 0; j < NT; j++) {
                const uint32_t h = u < 2 ? wd[buf][j].x : wd[buf][j].y;
                sb[j] = u16_to_f((uint16_t)((u & 1) ? h >> 16 : h & 0xffffu));
            }
#pragma unroll
            for (int i = 0; i < MT; i++)
#pragma unroll
                for (int j = 0; j < NT; j++) {
                    const intx4 ci = __builtin_amdgcn_mfma_i32_16x16x32_i8(ab[buf][i][u], wb[buf][j][u], intx4{0, 0, 0, 0}, 0, 0, 0);
                    floatx4 sa;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float4 a4 = ad[buf][i][r];
                        sa[r] = u == 0 ? a4.x : u == 1 ? a4.y : u == 2 ? a4.z : a4.w;
                    }
                    q8_scale_acc(acc[i][j], sb[j], sa, ci);
                }
        }
    };
    if constexpr (ALDS && CPW > 0) {   // every chunk of the wave in flight at once (gemm_skinny_kernel's CPW)
        static_assert(CPW <= 4, "the per-chunk vmcnt waits below are written out for at most 4 chunks");
        uint8_t *my = (uint8_t *)lds_raw + wid * (CPW * MT * 16 * 128);
        long wq[CPW][NT][4];
        uint2 wdq[CPW][NT];
        float4 adq[CPW][MT][4];
#pragma unroll
        for (int k = 0; k < CPW; k++) {
            const int c = wid + k * KW;
#pragma unroll
            for (int t = 0; t < NT; t++) {
#pragma unroll
                for (int u = 0; u < 4; u++) wq[k][t][u] = __builtin_nontemporal_load((const long *)(wrow[t] + c * 128 + u * 32));
                wdq[k][t] = *(const uint2 *)(wdrow[t] + c * 4);
            }
#pragma unroll
            for (int t = 0; t < MT; t++)
#pragma unroll
                for (int r = 0; r < 4; r++) adq[k][t][r] = *(const float4 *)(adrow[t][r] + c * 4);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int p = 0; p < MT * 2; p++) {   // 1 KiB = 8 rows of 128 B per piece
                const int r = p * 8 + (lane >> 3), ch = (lane & 7) ^ (r & 7);
                const int m = m0 + r;
                const int8_t *src = m < M ? g.Aq + (long)m * g.lda + c * 128 + ch * 16 : (const int8_t *)g_zero_line_s;
                __builtin_amdgcn_global_load_lds((glb_void_s *)src, (lds_void_s *)(my + k * (MT * 16 * 128) + p * 1024), 16, 0, 0);
            }
            asm volatile("" ::: "memory");   // chunk k's requests together, in chunk order (the waits below count them)
        }
        constexpr int PER = MT * 2 + NT * 5 + MT * 4;   // VMEM requests per chunk
#pragma unroll
        for (int k = 0; k < CPW; k++) {
            if (k == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW - 1) * PER)) : "memory");
            else if (k == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW > 1 ? CPW - 2 : 0) * PER)) : "memory");
            else if (k == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW > 2 ? CPW - 3 : 0) * PER)) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vmc((CPW > 3 ? CPW - 4 : 0) * PER)) : "memory");
            const uint8_t *mk = my + k * (MT * 16 * 128);
#pragma unroll
            for (int t = 0; t < NT; t++) {
#pragma unroll
                for (int u = 0; u < 4; u++) wb[0][t][u] = wq[k][t][u];
                wd[0][t] = wdq[k][t];
            }
#pragma unroll
            for (int t = 0; t < MT; t++) {
#pragma unroll
                for (int r = 0; r < 4; r++) ad[0][t][r] = adq[k][t][r];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int r = t * 16 + c16, b = 32 * u + 8 * q;
                    ab[0][t][u] = *(const long *)(mk + r * 128 + ((((b >> 4) ^ (r & 7)) << 4) | (b & 15)));
                }
            }
            mma(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if constexpr (ALDS) {
        uint8_t *my = (uint8_t *)lds_raw + wid * (MT * 16 * 128);
        for (int c = wid; c < nch; c += KW) {
#pragma unroll
            for (int p = 0; p < MT * 2; p++) {   // 1 KiB = 8 rows of 128 B per piece
                const int r = p * 8 + (lane >> 3), ch = (lane & 7) ^ (r & 7);
                const int m = m0 + r;
                const int8_t *src = m < M ? g.Aq + (long)m * g.lda + c * 128 + ch * 16 : (const int8_t *)g_zero_line_s;
                __builtin_amdgcn_global_load_lds((glb_void_s *)src, (lds_void_s *)(my + p * 1024), 16, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < NT; t++) {
#pragma unroll
                for (int u = 0; u < 4; u++) wb[0][t][u] = __builtin_nontemporal_load((const long *)(wrow[t] + c * 128 + u * 32));
                wd[0][t] = *(const uint2 *)(wdrow[t] + c * 4);
            }
#pragma unroll
            for (int t = 0; t < MT; t++)
#pragma unroll
                for (int r = 0; r < 4; r++) ad[0][t][r] = *(const float4 *)(adrow[t][r] + c * 4);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int t = 0; t < MT; t++)
#pragma unroll
                for (int u = 0; u < 4; u++) {   // bytes 32u + 8q .. +8 of row 16t + c16
                    const int r = t * 16 + c16, b = 32 * u + 8 * q;
                    ab[0][t][u] = *(const long *)(my + r * 128 + ((((b >> 4) ^ (r & 7)) << 4) | (b & 15)));
                }
            mma(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    } else {
        int c = wid;
        if (c < nch) load(0, c);
        for (; c < nch; c += 2 * KW) {
            if (c + KW < nch) load(1, c + KW);
            mma(0);
            if (c + KW >= nch) break;
            if (c + 2 * KW < nch) load(0, c + 2 * KW);
            mma(1);
        }
    }
    if constexpr (ALDS) __syncthreads();

#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NT; j++) red[wid][i * NT + j][lane] = acc[i][j];
    if constexpr (EPI == EPI_ARGMAX)
        if (tid < 64) rmax[tid] = 0ull;
    __syncthreads();
    epi.run(g, red, rmax, m0, n0, tid);
}

// grid: (column tiles, row blocks of 16*MT rows).  Blocks of one column tile
// are gridDim.x apart in dispatch order; with gridDim.x % 8 == 0 they share an
// XCD under the observed round-robin placement, so the weight tile's re-reads
// hit that XCD's L2 (speed only, never correctness).
// activations through LDS-DMA (VAR 4) unless the register-staged tiles are asked
// for: bit-identical (same fragments, same chunk order per wave), measured
// 16 % faster over a batch-64 layer's four projections (tools/skinny_bench.hip)
template <int MT, int NT, int KW, int EPI, int VAR>
static void run_skinny_v(const GemmArgs &g, hipStream_t s) {
    dim3 grid(g.N / (16 * NT), (g.M + 16 * MT - 1) / (16 * MT));
    const int cpw = (g.K >> 7) % KW == 0 && g.skinny_inflight ? (g.K >> 7) / KW : 0;   // whole chunks a wave: all in flight
    // (a CPW form is instantiated only where its chunk images fit the LDS: <= 128 KiB)
    constexpr int CH = KW * MT * 16 * 128 * 2;
    if (cpw == 1) hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, EPI, VAR, 1>), grid, dim3(64 * KW), 0, s, g);
    else if (cpw == 2 && 2 * CH <= 131072) hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, EPI, VAR, 2 * CH <= 131072 ? 2 : 1>), grid, dim3(64 * KW), 0, s, g);
    else if (cpw == 3 && 3 * CH <= 131072) hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, EPI, VAR, 3 * CH <= 131072 ? 3 : 1>), grid, dim3(64 * KW), 0, s, g);
    else hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, EPI, VAR>), grid, dim3(64 * KW), 0, s, g);
}
template <int MT, int NT, int KW, int EPI>
static void run_skinny(const GemmArgs &g, hipStream_t s) {
    if (g.regs_staged) hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, EPI, 0>), dim3(g.N / (16 * NT), (g.M + 16 * MT - 1) / (16 * MT)),
                                          dim3(64 * KW), 0, s, g);
    else if (g.wdef) run_skinny_v<MT, NT, KW, EPI, 4 | 8>(g, s);
    else run_skinny_v<MT, NT, KW, EPI, 4>(g, s);
}

template <int MT, int NT, int KW, int EPI>
static void run_skinny_q8(const GemmArgs &g, hipStream_t s) {
    dim3 grid(g.N / (16 * NT), (g.M + 16 * MT - 1) / (16 * MT));
    const int cpw = (g.K >> 7) % KW == 0 && g.skinny_inflight ? (g.K >> 7) / KW : 0;
    constexpr int CH = KW * MT * 16 * 128;
    if (g.regs_staged) hipLaunchKernelGGL((gemm_skinny_q8_kernel<MT, NT, KW, EPI, 0>), grid, dim3(64 * KW), 0, s, g);
    else if (cpw == 1) hipLaunchKernelGGL((gemm_skinny_q8_kernel<MT, NT, KW, EPI, 4, 1>), grid, dim3(64 * KW), 0, s, g);
    else if (cpw == 2 && 2 * CH <= 131072) hipLaunchKernelGGL((gemm_skinny_q8_kernel<MT, NT, KW, EPI, 4, 2 * CH <= 131072 ? 2 : 1>), grid, dim3(64 * KW), 0, s, g);
    else if (cpw == 3 && 3 * CH <= 131072) hipLaunchKernelGGL((gemm_skinny_q8_kernel<MT, NT, KW, EPI, 4, 3 * CH <= 131072 ? 3 : 1>), grid, dim3(64 * KW), 0, s, g);
    else hipLaunchKernelGGL((gemm_skinny_q8_kernel<MT, NT, KW, EPI, 4>), grid, dim3(64 * KW), 0, s, g);
}

template <int MTMAX, int NT, int KW, int EPI>
static void skinny_q8_mt(const GemmArgs &g, hipStream_t s) {
    const int mt = (g.M + 15) / 16;
    if (mt <= 1 || MTMAX == 1) run_skinny_q8<1, NT, KW, EPI>(g, s);
    else if (mt <= 2 || MTMAX == 2) run_skinny_q8<MTMAX >= 2 ? 2 : 1, NT, KW, EPI>(g, s);
    else if (mt <= 3 || MTMAX == 3) run_skinny_q8<MTMAX >= 3 ? 3 : 1, NT, KW, EPI>(g, s);
    else run_skinny_q8<MTMAX >= 4 ? 4 : 1, NT, KW, EPI>(g, s);
}

// MTMAX: rows per block cap (x16); smaller batches use the fewest tiles
template <int MTMAX, int NT, int KW, int EPI>
static void skinny_mt(const GemmArgs &g, hipStream_t s) {
    const int mt = (g.M + 15) / 16;
    if (mt <= 1 || MTMAX == 1) run_skinny<1, NT, KW, EPI>(g, s);
    else if (mt <= 2 || MTMAX == 2) run_skinny<MTMAX >= 2 ? 2 : 1, NT, KW, EPI>(g, s);
    else if (mt <= 3 || MTMAX == 3) run_skinny<MTMAX >= 3 ? 3 : 1, NT, KW, EPI>(g, s);
    else run_skinny<MTMAX >= 4 ? 4 : 1, NT, KW, EPI>(g, s);
}


bool launch_gemm_skinny(int epi, const GemmArgs &g, hipStream_t s) {
    const bool off = g.no_skinny != 0;
    if (off || g.M <= 0 || g.M > 128 || g.K % 128 != 0 || g.lda % 8 != 0 || g.ldw % 8 != 0) return false;
    switch (epi) {
        case EPI_F32:
        case EPI_F16:
            if (g.N % 16 != 0) return false;
            // tilings picked with tools/skinny_bench.hip at M = 64; 65..128 rows (round 5, M = 128,
            // us a launch): QKV 32-column tiles of 64 rows 9.55 -> 7.30, o / down 32-row blocks
            // 8.01 -> 6.14 / 12.64 -> 8.81 -- fewer activation re-reads per weight byte
            if (g.M > 64 && g.N >= 4096 && g.N % 32 == 0) {
                if (epi == EPI_F32) run_skinny<4, 2, 8, EPI_F32>(g, s); else run_skinny<4, 2, 8, EPI_F16>(g, s);
            } else if (g.M > 64) {
                if (epi == EPI_F32) run_skinny<2, 1, 8, EPI_F32>(g, s); else run_skinny<2, 1, 8, EPI_F16>(g, s);
            } else if (g.N >= 4096) {   // QKV: 256 column tiles, all rows per block, K over 8 waves
                if (epi == EPI_F32) skinny_mt<4, 1, 8, EPI_F32>(g, s); else skinny_mt<4, 1, 8, EPI_F16>(g, s);
            } else {             // o / down projections: 64 column tiles x 16-row blocks, K over 8 waves
                if (epi == EPI_F32) skinny_mt<1, 1, 8, EPI_F32>(g, s); else skinny_mt<1, 1, 8, EPI_F16>(g, s);
            }
            return true;
        case EPI_SWIGLU_F16:
        case EPI_SWIGLU_F32:
            if (g.N % 32 != 0) return false;
            // 33..64 rows: all of them in one row block, K over 8 waves (one chunk each at K = 1024):
            // every weight byte read once instead of once per 32-row block (tools/skinny_bench.hip,
            // 64 rows, 6144 x 1024: 9.31 -> 7.13 us a launch, round 5)
            // 65..128 rows: 64-row blocks of 64 columns, 12.95 -> 10.38 us at M = 128 (round 5)
            if (g.M > 64 && g.N % 64 == 0) {
                if (epi == EPI_SWIGLU_F16) run_skinny<4, 4, 8, EPI_SWIGLU_F16>(g, s); else run_skinny<4, 4, 8, EPI_SWIGLU_F32>(g, s);
            } else if (g.M > 32 && g.M <= 64) {
                if (epi == EPI_SWIGLU_F16) run_skinny<4, 2, 8, EPI_SWIGLU_F16>(g, s); else run_skinny<4, 2, 8, EPI_SWIGLU_F32>(g, s);
            } else if (epi == EPI_SWIGLU_F16) {
                skinny_mt<2, 2, 4, EPI_SWIGLU_F16>(g, s);
            } else {
                skinny_mt<2, 2, 4, EPI_SWIGLU_F32>(g, s);
            }
            return true;
        case EPI_ARGMAX:
            if (g.N % 64 != 0) return false;
            // (64-row x 128-column tiles and 4 K waves measured 136-186 us against
            // 139 for this one at batch 64: tools/experiments.sh lmh)
            skinny_mt<4, 4, 2, EPI_ARGMAX>(g, s);
            return true;
        default:
            return false;
    }
}

bool launch_gemm_skinny_q8(int epi, const GemmArgs &g, hipStream_t s) {
    const bool off = g.no_skinny != 0;
    if (off || g.M <= 0 || g.M > 128 || g.K % 128 != 0 || g.lda % 16 != 0 || g.ldw % 16 != 0 || g.ldad % 4 != 0) return false;
    switch (epi) {
        case EPI_F32:
            if (g.N % 16 != 0) return false;
            // QKV: all 64 rows a block (tools/skinny_q8_bench.hip, 64 rows: 7.18 -> 6.53 us a
            // launch with every chunk in flight; the same K split, so the same bits); o / down:
            // 16-row blocks (32- and 64-row blocks 1.3-3.7 us slower)
            // 65..128 rows (tools/skinny_q8_bench.hip at 128 rows): QKV 32-column tiles of 64
            // rows 9.17 -> 8.60 us, o / down 32-row blocks 8.97 -> 7.27 / 12.55 -> 9.42 us
            if (g.M > 64 && g.N >= 4096 && g.N % 32 == 0) run_skinny_q8<4, 2, 8, EPI_F32>(g, s);
            else if (g.M > 64) run_skinny_q8<2, 1, 8, EPI_F32>(g, s);
            else if (g.N >= 4096) skinny_q8_mt<4, 1, 8, EPI_F32>(g, s);
            else skinny_q8_mt<1, 1, 8, EPI_F32>(g, s);
            return true;
        case EPI_SWIGLU_F32:
            if (g.N % 32 != 0) return false;
            skinny_q8_mt<2, 2, 4, EPI_SWIGLU_F32>(g, s);
            return true;
        case EPI_SWIGLU_Q8:
            // 64-column blocks: 32 output columns, one Q8_0 block a row; K over 8 waves
            // (tools/skinny_q8_bench.hip, 64 rows: 10.16 us against 10.43 for the fp32
            // SwiGLU form alone, which the separate quantisation launch then followed)
            // (65..128 rows: 64-row blocks, 18.30 -> 12.52 us at 128 rows)
            if (g.N % 64 != 0 || !g.out_q || !g.out_d || g.ldoq % 32 != 0) return false;
            if (g.M > 64) run_skinny_q8<4, 4, 8, EPI_SWIGLU_Q8>(g, s);
            else skinny_q8_mt<2, 4, 8, EPI_SWIGLU_Q8>(g, s);
            return true;
        default:
            return false;
    }
}

}  // namespace qasr
