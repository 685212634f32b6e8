// lmhead.hip -- the decode-batch LM head in one launch (9 <= M <= 128 rows):
// final RMS norm + tied-embedding GEMM (151936 x 1024 f16) + first-index
// argmax + the greedy step's bookkeeping (src/text_decoder.cpp forward's last
// ggml_rms_norm / ggml_mul / ggml_mul_mat over model.output, then
// src/qwen3_asr.cpp:270-296's sample_greedy per sequence).
//
// The skinny GEMM (gemm_skinny.hip) took 140-150 us for these 311 MB: 2374
// workgroups each streamed 128 KB of weights but re-read the whole 64 x 1024
// activation (another 128 KB) through LDS-DMA, every 64-column tile folded its
// keys into the same 64 global argmax words (152k atomics on 64 addresses), and
// the norm, the key reset and the bookkeeping were five more launches.
//
// Here one persistent workgroup per CU normalises the rows once into LDS
// (rms_row's arithmetic: the values launch_rmsnorm_f16 writes), then each wave
// streams a contiguous run of 16-column units of the weight matrix through a
// D-deep ring of fragment registers (nontemporal buffer loads, out-of-range
// items read as zeros without a memory access), multiplies them against the
// LDS rows on v_mfma_f32_16x16x32_f16 (K ascending in 32-wide steps, fp32
// accumulation; even and odd chunks in two accumulators summed at the end, the
// order of gemm_skinny_kernel<4, 4, 2>'s two K waves, so the logits are
// bit-identical to the separate launches'), keeps a per-lane running best key per row across all its
// units, and reduces those once at the end: one atomicMax per row per
// workgroup, then the last workgroup decodes the tokens (tok, hist[step+1],
// pos += 1, n_kv += 1, step += 1) and re-arms amax / done (zero at rest).
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

namespace {

constexpr int LMH_K = 1024;   // hidden width this kernel is built for (host checks)
typedef __attribute__((address_space(3))) void lds_void_l;
typedef __attribute__((address_space(1))) void glb_void_l;

// LDS row layout: 128 chunks of 16 B per row, chunk ch stored at ch ^ (row & 15)
// so the 16 rows of a fragment read hit 16 distinct 16-B bank groups
__device__ __forceinline__ int lmh_off(int row, int k) {   // element offset of (row, k), k % 8 == 0 .. +7
    const int ch = k >> 3;
    return row * LMH_K + ((ch ^ (row & 15)) << 3) + (k & 7);
}

template <int MT, int WPG, int D>
__global__ __launch_bounds__(64 * WPG) void lmhead_batch_kernel(GemvArgs g) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];   // [MT*16][LMH_K] fp16, swizzled
    __shared__ unsigned long long bestk[WPG][MT * 16];
    __shared__ int last_wg, st;
    stamp_start(g.stamp);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int q = lane >> 4, c16 = lane & 15;
    const int M = g.M;

    // ---- this wave's units (16 weight rows each) and items (unit, 128-wide K chunk)
    const int U = g.N >> 4, TW = gridDim.x * WPG, gw = blockIdx.x * WPG + wid;
    const int u0 = (int)((long)gw * U / TW), u1 = (int)((long)(gw + 1) * U / TW);
    const int n_items = (u1 - u0) * (LMH_K / 128);
    const uint32_t wbytes = (uint32_t)((long)g.N * LMH_K * 2);
    const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc((void *)g.W, (short)0, (int)wbytes, 0x00020000);
    u32x4 wb[D][4];
    auto load = [&](int b, int j) {
        const int u = u0 + (j >> 3), c = j & 7;
        const uint32_t base = (uint32_t)(((long)(u * 16 + c16) * LMH_K + c * 128 + q * 8) * 2);
#pragma unroll
        for (int s = 0; s < 4; s++)
            wb[b][s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wsrd, j < n_items ? base + 64 * s : wbytes, 0, 2));
    };
#pragma unroll
    for (int b = 0; b < D; b++) load(b, b);

    // ---- prologue: rows -> RMS norm (rms_row<1024> arithmetic) -> fp16 LDS;
    //      the wave's rows in batches of RB, every load of a batch in flight
    //      together (one row at a time left the weight ring idle for ~10 us at 64 rows)
    constexpr int R = MT * 16 / WPG, RB = R < 4 ? R : 4;
    static_assert(R * WPG == MT * 16, "rows split evenly over the waves");
    float4 wv[4];
#pragma unroll
    for (int i = 0; i < 4; i++) wv[i] = *(const float4 *)(g.norm_w + 4 * lane + 256 * i);
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += RB) {
        float4 v[RB][4];
#pragma unroll
        for (int r = 0; r < RB; r++) {
            const int m = wid + WPG * (r0 + r);
            const float *xr = g.x + (long)(m < M ? m : 0) * g.ldx;
#pragma unroll
            for (int i = 0; i < 4; i++) v[r][i] = *(const float4 *)(xr + 4 * lane + 256 * i);
        }
#pragma unroll
        for (int r = 0; r < RB; r++) {
            const int m = wid + WPG * (r0 + r);
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 4; i++)
                s += ((double)fmul_rn(v[r][i].x, v[r][i].x) + (double)fmul_rn(v[r][i].y, v[r][i].y)) +
                     ((double)fmul_rn(v[r][i].z, v[r][i].z) + (double)fmul_rn(v[r][i].w, v[r][i].w));
            s = wave_sum_d(s);
            const float mean = (float)(s / LMH_K);
            const float scale = 1.0f / sqrtf(mean + g.eps);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uint32_t lo = f_to_u16(fmul_rn(fmul_rn(v[r][i].x, scale), wv[i].x)) |
                              ((uint32_t)f_to_u16(fmul_rn(fmul_rn(v[r][i].y, scale), wv[i].y)) << 16);
                uint32_t hi = f_to_u16(fmul_rn(fmul_rn(v[r][i].z, scale), wv[i].z)) |
                              ((uint32_t)f_to_u16(fmul_rn(fmul_rn(v[r][i].w, scale), wv[i].w)) << 16);
                if (m >= M) lo = hi = 0u;   // rows past M: zeros
                *(uint2 *)(xs + lmh_off(m, 4 * lane + 256 * i)) = make_uint2(lo, hi);
            }
        }
    }
    __syncthreads();

    // ---- stream: item j = (unit u0 + j / 8, K chunk j % 8), ring slot j % D
    unsigned long long best[MT][4];
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int r = 0; r < 4; r++) best[i][r] = 0ull;
    floatx4 acc[2][MT];   // even / odd K chunks: the skinny kernel's two K waves (bit-identical logits)
    const int nvalid = g.n_valid > 0 ? g.n_valid : g.N;
    for (int j0 = 0; j0 < n_items; j0 += D) {
#pragma unroll
        for (int b = 0; b < D; b++) {
            const int j = j0 + b;
            if (j >= n_items) break;
            const int c = j & 7;
            if (c == 0) {
#pragma unroll
                for (int i = 0; i < MT; i++) acc[0][i] = acc[1][i] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int s = 0; s < 4; s++) {
#pragma unroll
                for (int i = 0; i < MT; i++) {
                    const half8 a8 = *(const half8 *)(xs + lmh_off(i * 16 + c16, c * 128 + 32 * s + 8 * q));
                    acc[c & 1][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, __builtin_bit_cast(half8, wb[b][s]), acc[c & 1][i], 0, 0, 0);
                }
            }
            load(b, j + D);
            if (c == 7) {   // unit done: C layout, lane (q, c16) = rows 16i + 4q + r, column 16u + c16
                const int col = (u0 + (j >> 3)) * 16 + c16;
#pragma unroll
                for (int i = 0; i < MT; i++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = i * 16 + 4 * q + r;
                        const float v = acc[0][i][r] + acc[1][i][r];
                        if (g.out_f32 && row < M) g.out_f32[(long)row * g.ldo + col] = v;
                        const unsigned long long key = col < nvalid ? argmax_key(v, col) : 0ull;
                        best[i][r] = key > best[i][r] ? key : best[i][r];
                    }
            }
        }
    }

    // ---- per-row best over the 16 columns lanes, the waves, then the workgroups
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            unsigned long long k = best[i][r];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const unsigned long long t = __shfl_xor(k, o, 64);
                k = t > k ? t : k;
            }
            if (c16 == 0) bestk[wid][i * 16 + 4 * q + r] = k;
        }
    __syncthreads();
    if (tid < M) {
        unsigned long long b = bestk[0][tid];
#pragma unroll
        for (int w = 1; w < WPG; w++) b = bestk[w][tid] > b ? bestk[w][tid] : b;
        const unsigned long long old = atomicMax(g.amax + tid, b);
        asm volatile("" ::"v"(old));   // returned value used: the max has been performed at L2
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) last_wg = __hip_atomic_fetch_add(g.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (last_wg) {
        if (tid == 0) st = *g.step;
        __syncthreads();
        if (tid < M) {
            const unsigned long long k = __hip_atomic_load(g.amax + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int id = argmax_key_idx(k);
            g.tok_out[tid] = id;
            if (g.hist) g.hist[(long)tid * g.hist_stride + st + 1] = id;
            g.pos[tid] += 1;
            if (g.nkv) g.nkv[tid] += 1;
            __hip_atomic_store(g.amax + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0) {
            if (!g.keep_step) *g.step = st + 1;
            __hip_atomic_store(g.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    stamp_end(g.stamp);
}

// 8 waves a CU with a 4-deep ring (tools/micro/lmh_bench.hip, MI355X: 16 rows
// 60.8 us against 68.9 with 16 waves x 3; 64 rows: 6- and 8-deep rings and 4
// waves x 8 or 12 slower)
template <int MT, int WPG = 8, int D = 4>
void run_lmhead(const GemvArgs &g, hipStream_t s) {
    static int ncu_dev[64];   // per device: CU count once the LDS attribute is set
    int dev = 0;
    (void)hipGetDevice(&dev);
    int &ncu = ncu_dev[dev & 63];
    if (!ncu) {
        int n = 0;
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipFuncSetAttribute((const void *)lmhead_batch_kernel<MT, WPG, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  MT * 16 * LMH_K * 2);
        ncu = n > 0 ? n : 256;
    }
    hipLaunchKernelGGL((lmhead_batch_kernel<MT, WPG, D>), dim3(ncu), dim3(64 * WPG), MT * 16 * LMH_K * 2, s, g);
}

// ---- 65..128 rows in one launch, the embedding read once (round 6).  The
// 128 normalised rows (256 KB fp16) do not fit the LDS, so they live in
// registers: wave w holds rows 16w .. 16w + 15 as its 32 MFMA A fragments of
// K (128 VGPRs a lane), staged through LDS 32 rows at a time with
// lmhead_batch_kernel's norm arithmetic.  The weight units (16 vocabulary rows
// x 1024, 32 KB) stream through an L128_R-slot LDS ring by LDS-DMA
// (nontemporal, 16-B chunks XOR-swizzled by row so the fragment reads of 16
// rows hit distinct banks), two units in flight behind the one being read,
// and every unit is read by all eight waves: one HBM read of the 311 MB
// embedding per step instead of one per 64-row half.  Per (row tile, unit)
// the MFMA order is lmhead_batch_kernel's -- K chunks ascending, even / odd
// chunks in two accumulators summed at the end -- so the logits, and the
// tokens, are bit-identical to the two-launch path (tools/micro/lmh128_bench).
// Each wave owns its rows outright: per row one atomicMax per workgroup, then
// the last workgroup decodes the tokens as lmhead_batch_kernel does.  (A
// 9-slot ring of half units, seven in flight, ran slower: 97 against 86 us,
// profiles/r6/lmhead128_r9ring_ab.txt -- twice the barriers.)
constexpr int L128_R = 4;                  // ring slots (32 KB each)
constexpr int L128_UNIT = 16 * LMH_K;      // halves per unit
constexpr int L128_LDS = L128_R * L128_UNIT * 2;

__global__ __launch_bounds__(512) void lmhead128_kernel(GemvArgs g) {
    extern __shared__ __attribute__((aligned(16))) uint16_t ring[];   // [L128_R][16][LMH_K], swizzled
    __shared__ int last_wg, st;
    stamp_start(g.stamp);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = lane >> 4, c16 = lane & 15;
    const int M = g.M;
    const int U = g.N >> 4;
    const int u0 = (int)((long)blockIdx.x * U / gridDim.x), u1 = (int)((long)(blockIdx.x + 1) * U / gridDim.x);
    const int nu = u1 - u0;
    // unit j of this workgroup -> ring slot j % R: 32 pieces of 1 KB (row r = piece / 2), four per wave
    auto issue = [&](int j) {
        const int u = u0 + j;
        uint16_t *dst = ring + (j % L128_R) * L128_UNIT;
#pragma unroll
        for (int ii = 0; ii < 4; ii++) {
            const int i = wid * 4 + ii, r = i >> 1, p = ((i & 1) << 6) + lane;
            const uint16_t *src = g.W + ((long)(u * 16 + r) * LMH_K + ((p ^ (r & 15)) << 3));
            __builtin_amdgcn_global_load_lds((glb_void_l *)src, (lds_void_l *)(dst + i * 512), 16, 0, 2);
        }
    };
    // units 0, 1 land while the rows are normalised (slots 2, 3 hold the staging rows meanwhile)
    if (nu > 0) issue(0);
    if (nu > 1) issue(1);

    // ---- prologue: rows 32p .. 32p + 31 -> RMS norm -> fp16 staging (slots 2-3), then the two
    //      waves owning them take their A fragments; wave w normalises rows 32p + w + 8i
    uint16_t *xs = ring + 2 * L128_UNIT;   // [32][LMH_K], lmh_off swizzle
    half8 af[32];                          // K step t: k = 32 t + 8 q .. + 8 of row 16 wid + c16
    float4 wv[4];
#pragma unroll
    for (int i = 0; i < 4; i++) wv[i] = *(const float4 *)(g.norm_w + 4 * lane + 256 * i);
#pragma unroll
    for (int p = 0; p < 4; p++) {
        float4 v[4][4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int m = 32 * p + wid + 8 * r;
            const float *xr = g.x + (long)(m < M ? m : 0) * g.ldx;
#pragma unroll
            for (int i = 0; i < 4; i++) v[r][i] = *(const float4 *)(xr + 4 * lane + 256 * i);
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int m = 32 * p + wid + 8 * r, lr = wid + 8 * r;
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 4; i++)
                s += ((double)fmul_rn(v[r][i].x, v[r][i].x) + (double)fmul_rn(v[r][i].y, v[r][i].y)) +
                     ((double)fmul_rn(v[r][i].z, v[r][i].z) + (double)fmul_rn(v[r][i].w, v[r][i].w));
            s = wave_sum_d(s);
            const float mean = (float)(s / LMH_K);
            const float scale = 1.0f / sqrtf(mean + g.eps);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uint32_t lo = f_to_u16(fmul_rn(fmul_rn(v[r][i].x, scale), wv[i].x)) |
                              ((uint32_t)f_to_u16(fmul_rn(fmul_rn(v[r][i].y, scale), wv[i].y)) << 16);
                uint32_t hi = f_to_u16(fmul_rn(fmul_rn(v[r][i].z, scale), wv[i].z)) |
                              ((uint32_t)f_to_u16(fmul_rn(fmul_rn(v[r][i].w, scale), wv[i].w)) << 16);
                if (m >= M) lo = hi = 0u;   // rows past M: zeros
                *(uint2 *)(xs + lmh_off(lr, 4 * lane + 256 * i)) = make_uint2(lo, hi);
            }
        }
        __syncthreads();
        if ((wid >> 1) == p) {
            const int lr = 16 * (wid & 1) + c16;
#pragma unroll
            for (int t = 0; t < 32; t++) af[t] = *(const half8 *)(xs + lmh_off(lr, 32 * t + 8 * q));
        }
        __syncthreads();
    }
    if (nu > 2) issue(2);

    // ---- stream: unit j from slot j % R; unit j + R - 1 issued once every wave is past unit j - 1
    unsigned long long best[4] = {0ull, 0ull, 0ull, 0ull};
    const int nvalid = g.n_valid > 0 ? g.n_valid : g.N;
    for (int j = 0; j < nu; j++) {
        // this wave's pieces of unit j landed: the units after it still in flight (four pieces each)
        const int later = min(nu - 1 - j, L128_R - 2);
        if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // every wave's pieces of unit j; every wave done with unit j - 1 (its slot is free)
        if (j + L128_R - 1 < nu) issue(j + L128_R - 1);
        const uint16_t *sl = ring + (j % L128_R) * L128_UNIT + c16 * LMH_K;
        floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++) {
                const int ch = 16 * c + 4 * s4 + q;
                const half8 b8 = *(const half8 *)(sl + ((ch ^ c16) << 3));
                acc[c & 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[4 * c + s4], b8, acc[c & 1], 0, 0, 0);
            }
        const int col = (u0 + j) * 16 + c16;
#pragma unroll
        for (int r = 0; r < 4; r++) {   // C layout: lane (q, c16) = rows 16 wid + 4q + r, column col
            const int row = 16 * wid + 4 * q + r;
            const float v = acc[0][r] + acc[1][r];
            if (g.out_f32 && row < M) g.out_f32[(long)row * g.ldo + col] = v;
            const unsigned long long key = col < nvalid ? argmax_key(v, col) : 0ull;
            best[r] = key > best[r] ? key : best[r];
        }
    }

    // ---- per-row best over the 16 column lanes; each row belongs to one wave
#pragma unroll
    for (int r = 0; r < 4; r++) {
        unsigned long long k = best[r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const unsigned long long t = __shfl_xor(k, o, 64);
            k = t > k ? t : k;
        }
        const int row = 16 * wid + 4 * q + r;
        if (c16 == 0 && row < M) {
            const unsigned long long old = atomicMax(g.amax + row, k);
            asm volatile("" ::"v"(old));   // returned value used: the max has been performed at L2
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) last_wg = __hip_atomic_fetch_add(g.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (last_wg) {
        if (tid == 0) st = *g.step;
        __syncthreads();
        if (tid < M) {
            const unsigned long long k = __hip_atomic_load(g.amax + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int id = argmax_key_idx(k);
            g.tok_out[tid] = id;
            if (g.hist) g.hist[(long)tid * g.hist_stride + st + 1] = id;
            g.pos[tid] += 1;
            if (g.nkv) g.nkv[tid] += 1;
            __hip_atomic_store(g.amax + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0) {
            if (!g.keep_step) *g.step = st + 1;
            __hip_atomic_store(g.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    stamp_end(g.stamp);
}

void run_lmhead128(const GemvArgs &g, hipStream_t s) {
    static int ncu_dev[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    int &ncu = ncu_dev[dev & 63];
    if (!ncu) {
        int n = 0;
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipFuncSetAttribute((const void *)lmhead128_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, L128_LDS);
        ncu = n > 0 ? n : 256;
    }
    hipLaunchKernelGGL(lmhead128_kernel, dim3(ncu), dim3(512), L128_LDS, s, g);
}

}  // namespace

bool launch_lmhead_batch(const GemvArgs &g, hipStream_t s) {
    if (g.M < 1 || g.M > 128 || g.K != LMH_K || g.N % 16 != 0 || !g.x || !g.norm_w || !g.amax || !g.done || !g.tok_out ||
        !g.step || !g.pos || g.Wd)
        return false;
    if (g.M > 64) {   // 65..128 rows: the rows in registers, the embedding read once (round 6; until then one
                      // launch per 64-row half, each streaming all 311 MB: tools/micro/lmh128_bench)
        run_lmhead128(g, s);
        return true;
    }
    const int mt = (g.M + 15) / 16;
    if (mt == 1) run_lmhead<1>(g, s);
    else if (mt == 2) run_lmhead<2>(g, s);
    else if (mt == 3) run_lmhead<3>(g, s);
    else run_lmhead<4>(g, s);
    return true;
}

}  // namespace qasr
