// elementwise.hip -- memory-bound kernels: conv1, norms, embedding/splice,
// argmax finish and decode-step bookkeeping.
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

// ------------------------------------------------------------------ conv1
// src/audio_encoder.cpp:105-112: ggml_conv_2d(1 -> C) = im2col(fp16) x fp16
// kernel.  K = 9 is below ggml's SIMD step, so ggml's vec_dot_f16 sums the 9
// exact fp16 products in double (its scalar leftover loop); we do the same.
// One wave per CONV1_ROWS consecutive output positions; lane l owns output
// channels 8l .. 8l+7 (its 72 fp16 weights and 8 biases stay in registers).
// The rows' 9-tap inputs are fetched by one load per lane (lane 9r + t: tap t
// of row r) and broadcast by v_readlane, so every row's loads are in flight at
// once; the rows' GELU-table gathers likewise, before the 16-byte NHWC stores
// (one dependent load / gather / store round per row measured 0.9 TB/s of
// output).  The same operations per output, so the same bits.  64 x 30 s
// (tools/micro/conv1_bench.hip, 5.9 GB of output): one row a round 5.77 ms;
// batched 2 / 4 / 6 / 7 rows 5.34 / 4.37 / 4.11 / 3.94 ms (7: 63 tap lanes, the
// most one wave holds); without the GELU gather 3.0 ms, and with each product as a
// double FMA over double weights (half the FP64 ops) 4.11 -- neither the gather
// nor the FP64 sums alone bound it.
#ifndef CONV1_ROWS
#define CONV1_ROWS 7
#endif
__global__ __launch_bounds__(256) void conv1_kernel(const float *__restrict__ mel, const ChunkDesc *__restrict__ chunks,
                                                    const int *__restrict__ row1_start, int n_chunks, int rows1,
                                                    const uint16_t *__restrict__ w, const float *__restrict__ b,
                                                    const uint16_t *__restrict__ lut, int C, uint16_t *__restrict__ act1) {
    static_assert(9 * CONV1_ROWS <= 64, "one tap per lane");
    // grid (positions / 16, chunk): no row -> chunk search
    const ChunkDesc cd = chunks[blockIdx.y];
    const int nloc = 64 * cd.W1;
    const int loc0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * CONV1_ROWS;
    const int lane = threadIdx.x & 63;
    if (loc0 >= nloc) return;   // wave-uniform
    float tap = 0.0f;
    if (lane < 9 * CONV1_ROWS) {
        const int r = lane / 9, t = lane - r * 9, kh = t / 3, kw = t - kh * 3;
        const int local = loc0 + r;
        if (local < nloc) {
            const int oh = local / cd.W1, ow = local - oh * cd.W1;
            const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;   // ih: mel bin, iw: frame in chunk
            if (ih >= 0 && ih < 128 && iw >= 0 && iw < cd.Lv) tap = mel[cd.mel_off + (long)ih * cd.T + iw];
        }
        tap = h2f(f2h(tap));
    }
    const bool active = lane * 8 < C;
    const int oc0 = active ? lane * 8 : 0;
    float wf[8][9];
    {
        const u32x4 *wp = (const u32x4 *)(w + oc0 * 9);   // 72 consecutive halves
        uint16_t wh[72];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const u32x4 v = wp[i];
#pragma unroll
            for (int e = 0; e < 4; e++) { wh[8 * i + 2 * e] = v[e] & 0xffffu; wh[8 * i + 2 * e + 1] = v[e] >> 16; }
        }
#pragma unroll
        for (int o = 0; o < 8; o++)
#pragma unroll
            for (int t = 0; t < 9; t++) wf[o][t] = u16_to_f(wh[o * 9 + t]);
    }
    const float4 b0 = *(const float4 *)(b + oc0), b1 = *(const float4 *)(b + oc0 + 4);
    const float bias[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    uint32_t hv[CONV1_ROWS][8];
#pragma unroll
    for (int r = 0; r < CONV1_ROWS; r++) {
        float in[9];
#pragma unroll
        for (int t = 0; t < 9; t++) in[t] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tap), r * 9 + t));
#pragma unroll
        for (int o = 0; o < 8; o++) {
            double sd = 0.0;
#pragma unroll
            for (int t = 0; t < 9; t++) sd += (double)(in[t] * wf[o][t]);
            hv[r][o] = gelu_lut_bits(fadd_rn((float)sd, bias[o]), lut);
        }
    }
#pragma unroll
    for (int r = 0; r < CONV1_ROWS; r++) {
        const int local = loc0 + r;
        if (!active || local >= nloc) continue;
        const u32x4 v = {hv[r][0] | hv[r][1] << 16, hv[r][2] | hv[r][3] << 16, hv[r][4] | hv[r][5] << 16, hv[r][6] | hv[r][7] << 16};
        *(u32x4 *)(act1 + (long)(cd.row1 + local) * C + oc0) = v;
    }
}

void launch_conv1(const float *mel, const ChunkDesc *chunks, const int *row1_start, int n_chunks, int rows1,
                  const uint16_t *w, const float *b, const uint16_t *gelu, int C, uint16_t *act1, hipStream_t s, int max_w1) {
    if (rows1 <= 0) return;
    const int per_block = 4 * CONV1_ROWS;
    const int max_loc = 64 * max_w1;   // the widest chunk's conv1 outputs (100-frame chunks: W1 = 50)
    hipLaunchKernelGGL(conv1_kernel, dim3((max_loc + per_block - 1) / per_block, n_chunks), dim3(256), 0, s, mel, chunks,
                       row1_start, n_chunks, rows1, w, b, gelu, C, act1);
}

// ------------------------------------------------------------------ norms
// ggml_norm: mean and centred variance summed in double, scale = 1/sqrtf(var+eps);
// then ggml_mul(w), ggml_add(b) as separately rounded fp32 ops; output rounded
// to fp16 (what the following ggml_mul_mat does to its input).
template <int D>
__global__ __launch_bounds__(256) void layernorm_kernel(const float *__restrict__ x, int M, const float *__restrict__ w,
                                                        const float *__restrict__ b, float eps, uint16_t *__restrict__ y,
                                                        float *__restrict__ y32) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    constexpr int PER = (D + 63) / 64;
    const float *xr = x + (long)row * D;
    float v[PER], wv[PER], bv[PER];
    // w / b requested with x (from x's own row when absent: the value is then unused),
    // so the stores below have no load between them (a load there made each store wait
    // for the previous one's write: round 6, as the GEMM epilogues)
    const float *wp = w ? w : xr, *bp = b ? b : xr;
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int k = lane + 64 * i;
        v[i] = k < D ? xr[k] : 0.0f;
        wv[i] = k < D ? wp[k] : 0.0f;
        bv[i] = k < D ? bp[k] : 0.0f;
        s += (double)v[i];
    }
    s = wave_sum_d(s);
    const float mean = (float)(s / D);
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int k = lane + 64 * i;
        if (k < D) {
            v[i] = fsub_rn(v[i], mean);
            s2 += (double)fmul_rn(v[i], v[i]);
        }
    }
    s2 = wave_sum_d(s2);
    const float var = (float)(s2 / D);
    const float scale = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int k = lane + 64 * i;
        if (k < D) {
            float t = fmul_rn(v[i], scale);
            if (w) t = fmul_rn(t, wv[i]);
            if (b) t = fadd_rn(t, bv[i]);
            if (y32) y32[(long)row * D + k] = t;
            else y[(long)row * D + k] = f_to_u16(t);
        }
    }
}

void launch_layernorm_f16(const float *x, int M, int D, const float *w, const float *b, float eps, uint16_t *y, hipStream_t s,
                          float *y32) {
    if (M <= 0) return;
    dim3 grid((M + 3) / 4);
    switch (D) {
        case 896: hipLaunchKernelGGL(layernorm_kernel<896>, grid, dim3(256), 0, s, x, M, w, b, eps, y, y32); break;
        case 256: hipLaunchKernelGGL(layernorm_kernel<256>, grid, dim3(256), 0, s, x, M, w, b, eps, y, y32); break;
        case 1024: hipLaunchKernelGGL(layernorm_kernel<1024>, grid, dim3(256), 0, s, x, M, w, b, eps, y, y32); break;
        default: hipLaunchKernelGGL(layernorm_kernel<2048>, grid, dim3(256), 0, s, x, M, w, b, eps, y, y32); break;
    }
}

// ggml_rms_norm: sum of squares (fp32 products) in double; scale = 1/sqrtf(mean+eps)
template <int D>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const float *__restrict__ x, int ldx, const int *__restrict__ row_idx, int M,
                                                      const float *__restrict__ w, float eps, uint16_t *__restrict__ y,
                                                      float *__restrict__ y32, int8_t *__restrict__ yq, float *__restrict__ yd) {
    // one wave per row; lane owns columns 4*lane + 256*i (16-B loads/stores).
    // yq/yd: Q8_0 output (int8 + fp32 block scales) of the same fp32 values,
    // a 32-block = 8 lanes
    static_assert(D % 256 == 0, "D must be a multiple of 256");
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    constexpr int PER = D / 256;
    const int src = row_idx ? row_idx[row] : row;
    const float *xr = x + (long)src * ldx;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) v[i] = *(const float4 *)(xr + 4 * lane + 256 * i);
    rms_row<D>(v, w, eps, row, y, y32, yq, yd);
}

static void rmsnorm_any(const float *x, int ldx, const int *row_idx, int M, int D, const float *w, float eps, uint16_t *y,
                        float *y32, int8_t *yq, float *yd, hipStream_t s) {
    if (M <= 0) return;
    dim3 grid((M + 3) / 4);
    switch (D) {
        case 1024: hipLaunchKernelGGL(rmsnorm_kernel<1024>, grid, dim3(256), 0, s, x, ldx, row_idx, M, w, eps, y, y32, yq, yd); break;
        case 256: hipLaunchKernelGGL(rmsnorm_kernel<256>, grid, dim3(256), 0, s, x, ldx, row_idx, M, w, eps, y, y32, yq, yd); break;
        default: hipLaunchKernelGGL(rmsnorm_kernel<2048>, grid, dim3(256), 0, s, x, ldx, row_idx, M, w, eps, y, y32, yq, yd); break;
    }
}

void launch_rmsnorm_f16(const float *x, int ldx, const int *row_idx, int M, int D, const float *w, float eps, uint16_t *y,
                        hipStream_t s, float *y32) {
    rmsnorm_any(x, ldx, row_idx, M, D, w, eps, y, y32, nullptr, nullptr, s);
}

void launch_rmsnorm_q8(const float *x, int ldx, int M, int D, const float *w, float eps, int8_t *yq, float *yd, hipStream_t s) {
    rmsnorm_any(x, ldx, nullptr, M, D, w, eps, nullptr, nullptr, yq, yd, s);
}

// --------------------------------------------------------- embedding/splice
__global__ __launch_bounds__(256) void embed_kernel(const int32_t *__restrict__ ids, int rows, const uint16_t *__restrict__ embd,
                                                    int hidden, const float *__restrict__ audio,
                                                    const int *__restrict__ row_audio, float *__restrict__ x) {
    const int row = blockIdx.x;
    if (row >= rows) return;
    const int ar = row_audio ? row_audio[row] : -1;
    float *dst = x + (long)row * hidden;
    if (ar >= 0) {
        const float *srcp = audio + (long)ar * hidden;
        for (int k = threadIdx.x; k < hidden; k += 256) dst[k] = srcp[k];
    } else {
        const uint16_t *srcp = embd + (long)ids[row] * hidden;
        for (int k = threadIdx.x; k < hidden; k += 256) dst[k] = u16_to_f(srcp[k]);
    }
}

void launch_embed(const int32_t *ids, int rows, const uint16_t *embd, int hidden, const float *audio, const int *row_audio,
                  float *x, hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(embed_kernel, dim3(rows), dim3(256), 0, s, ids, rows, embd, hidden, audio, row_audio, x);
}

// ------------------------------------------------------------ argmax etc.
__global__ void argmax_finish_kernel(const unsigned long long *__restrict__ amax, int B, int32_t *__restrict__ ids,
                                     int32_t *__restrict__ hist, int hist_stride, const int *__restrict__ step) {
    const int b = threadIdx.x;
    if (b >= B) return;
    const int id = argmax_key_idx(amax[b]);
    ids[b] = id;
    if (hist) hist[(long)b * hist_stride + *step] = id;
}

void launch_argmax_finish(const unsigned long long *amax, int B, int32_t *ids, int32_t *hist, int hist_stride, const int *step,
                          hipStream_t s) {
    hipLaunchKernelGGL(argmax_finish_kernel, dim3(1), dim3(256), 0, s, amax, B, ids, hist, hist_stride, step);
}

// dst row r = src row idx[r] (fp32 rows of D floats, 16-B lanes)
__global__ __launch_bounds__(256) void gather_rows_kernel(const float *__restrict__ src, const int *__restrict__ idx, int rows, int D,
                                                          float *__restrict__ dst) {
    const int per = D / 4;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)rows * per) return;
    const int r = (int)(i / per), c = (int)(i - (long)r * per);
    *(float4 *)(dst + (long)r * D + 4 * c) = *(const float4 *)(src + (long)idx[r] * D + 4 * c);
}
void launch_gather_rows(const float *src, const int *idx, int rows, int D, float *dst, hipStream_t s) {
    if (rows <= 0) return;
    const long n = (long)rows * (D / 4);
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, idx, rows, D, dst);
}

__global__ void fill_u64_kernel(unsigned long long *p, int n, unsigned long long v) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = v;
}

void launch_fill_u64(unsigned long long *p, int n, unsigned long long v, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(fill_u64_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, n, v);
}

__global__ void step_advance_kernel(int *row_pos, int *n_kv, int *step, int B) {
    const int b = threadIdx.x;
    if (b < B) {
        row_pos[b] += 1;
        n_kv[b] += 1;
    }
    if (b == 0) *step += 1;
}

void launch_step_advance(int *row_pos, int *n_kv, int *step, int B, hipStream_t s) {
    hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(256), 0, s, row_pos, n_kv, step, B);
}

// ------------------------------------------------------- Q8_0 activations
// ggml quantize_row_q8_0, x86 AVX2 path (ggml-cpu/arch/x86/quants.c): per
// 32 values amax, d = amax/127 (stored fp16), q = round-half-even(x * 127/amax).
// One thread per block; the fp16-rounded d is kept as fp32 for the dot.
__global__ __launch_bounds__(256) void quantize_q8_kernel(const float *__restrict__ x32, const uint16_t *__restrict__ x16, int ldx,
                                                          int M, int K, int gC, int8_t *__restrict__ q, float *__restrict__ d) {
    const int nb = K / 32;
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    if (t >= (long)M * nb) return;
    const int row = (int)(t / nb), b = (int)(t - (long)row * nb);
    float v[32];
    float amax = 0.0f;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const int j = 32 * b + i;
        const int col = gC > 0 ? (j & 15) * gC + (j >> 4) : j;
        v[i] = x32 ? x32[(long)row * ldx + col] : u16_to_f(x16[(long)row * ldx + col]);
        amax = fmaxf(amax, fabsf(v[i]));
    }
    d[(long)row * nb + b] = u16_to_f(f_to_u16(amax / 127.f));
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t u = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) u |= (uint32_t)(uint8_t)(int8_t)__builtin_rintf(fmul_rn(v[4 * i + e], id)) << (8 * e);
        w[i] = u;
    }
    u32x4 *dst = (u32x4 *)(q + (long)row * K + 32 * b);
    dst[0] = u32x4{w[0], w[1], w[2], w[3]};
    dst[1] = u32x4{w[4], w[5], w[6], w[7]};
}

// the same quantisation for dense rows, coalesced: lane = 4 consecutive values
// (one 16-B load), a 32-block = 8 lanes, a wave = 256 values of one row
__global__ __launch_bounds__(256) void quantize_q8_rows_kernel(const float *__restrict__ x32, const uint16_t *__restrict__ x16,
                                                               int ldx, int M, int K, int8_t *__restrict__ q, float *__restrict__ d) {
    const int wpr = K / 256;   // waves per row
    const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= (long)M * wpr) return;
    const int lane = threadIdx.x & 63;
    const int row = (int)(w / wpr), col = (int)(w - (long)row * wpr) * 256 + 4 * lane;
    float4 v;
    if (x32) {
        v = *(const float4 *)(x32 + (long)row * ldx + col);
    } else {
        const uint2 h = *(const uint2 *)(x16 + (long)row * ldx + col);
        v = make_float4(u16_to_f(h.x & 0xffffu), u16_to_f(h.x >> 16), u16_to_f(h.y & 0xffffu), u16_to_f(h.y >> 16));
    }
    float am = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    am = fmaxf(am, __shfl_xor(am, 4, 64));
    *(uint32_t *)(q + (long)row * K + col) = (uint32_t)(uint8_t)q8_quant(v.x, am) | (uint32_t)(uint8_t)q8_quant(v.y, am) << 8 |
                                            (uint32_t)(uint8_t)q8_quant(v.z, am) << 16 | (uint32_t)(uint8_t)q8_quant(v.w, am) << 24;
    if ((lane & 7) == 0) d[(long)row * (K / 32) + col / 32] = q8_scale(am);
}

void launch_quantize_q8(const float *x32, const uint16_t *x16, int ldx, int M, int K, int gather_C, int8_t *q, float *d,
                        hipStream_t s) {
    if (gather_C == 0 && K % 256 == 0 && ldx % 4 == 0 && M > 0) {
        const long waves = (long)M * (K / 256);
        hipLaunchKernelGGL(quantize_q8_rows_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, x32, x16, ldx, M, K, q, d);
        return;
    }
    const long n = (long)M * (K / 32);
    if (n <= 0) return;
    hipLaunchKernelGGL(quantize_q8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x32, x16, ldx, M, K, gather_C, q, d);
}

}  // namespace qasr
