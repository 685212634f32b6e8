// attention.hip -- encoder and decoder attention kernels for gfx950.
//
// Encoder (src/audio_encoder.cpp:466-486): full bidirectional attention per
// clip, 14 heads x 64, computed by the reference in fp32 (ggml_mul_mat on F32
// views, ggml_soft_max_ext).  Here: flash-style online softmax with exact-f32
// MFMA (v_mfma_f32_16x16x4_f32 = bitwise fp32 fma chain), swapped product
// S^T = K Q^T so each lane owns one query column and its softmax statistics
// are lane-local (reductions only across the 4 lane groups).
//
// Decoder prefill (src/text_decoder.cpp:534-540, ggml_flash_attn_ext CPU
// path): Q rounded to fp16, fp16 K/V cache, fp32 scores/softmax, causal, GQA
// 16 -> 8.  fp16 MFMA 16x16x32, same swapped layout; P.V consumes P straight
// from the accumulator registers through a k-index permutation.
//
// Decoder single token: split-K flash decoding (VALU; 2 q heads per kv head)
// + a combine kernel.
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

// ============================================================ encoder (fp32)
#define EKS 66   // K tile row stride (floats): conflict-free A reads
#define EVS 68   // V tile row stride (floats): conflict-free permuted reads

__global__ __launch_bounds__(256) void enc_attn_kernel(const float *__restrict__ qkv, const int *__restrict__ seg_start,
                                                       const int *__restrict__ seg_len, int D, uint16_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float Ks[64 * EKS];
    __shared__ __attribute__((aligned(16))) float Vs[64 * EVS];
    const int b = blockIdx.z, h = blockIdx.y;
    const int N = seg_len[b], r0 = seg_start[b];
    const int qblk = blockIdx.x * 64;
    if (qblk >= N) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, ql = lane & 15;
    const int ld = 3 * D;
    const int q = qblk + wid * 16 + ql;          // this lane's query
    const float scale = 0.125f;                  // 1/sqrt(64)
    // B operand of S^T = K Q^T: lane holds Q[q][4s + g]
    float qf[16];
#pragma unroll
    for (int s = 0; s < 16; s++) qf[s] = q < N ? qkv[(long)(r0 + q) * ld + h * 64 + 4 * s + g] : 0.0f;
    floatx4 o[4];
#pragma unroll
    for (int d = 0; d < 4; d++) o[d] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.0f;

    for (int k0 = 0; k0 < N; k0 += 64) {
        __syncthreads();
        // stage K and V tiles (64 keys x 64 dims fp32)
        for (int i = tid; i < 64 * 16; i += 256) {
            const int key = i >> 4, c4 = (i & 15) * 4;
            float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
            if (k0 + key < N) {
                const float *rowp = qkv + (long)(r0 + k0 + key) * ld + h * 64 + c4;
                kv = *(const float4 *)(rowp + D);
                vv = *(const float4 *)(rowp + 2 * D);
            }
            float *kd = Ks + key * EKS + c4;
            *(float2 *)kd = make_float2(kv.x, kv.y);
            *(float2 *)(kd + 2) = make_float2(kv.z, kv.w);
            *(float4 *)(Vs + key * EVS + c4) = vv;
        }
        __syncthreads();
        // S^T tiles: 4 key sub-tiles x 16 d-steps
        floatx4 st[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            st[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 16; s++) {
                const float a = Ks[(t * 16 + ql) * EKS + 4 * s + g];
                st[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[s], st[t], 0, 0, 0);
            }
        }
        // lane holds S[q][key = k0 + t*16 + 4g + i]
        float tmax = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int key = k0 + t * 16 + 4 * g + i;
                float v = st[t][i] * scale;
                if (key >= N) v = -INFINITY;
                st[t][i] = v;
                tmax = fmaxf(tmax, v);
            }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = expf(m_run - m_new);
        float psum = 0.0f;
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float p = expf(st[t][i] - m_new);
                st[t][i] = p;
                psum += p;
            }
        psum += __shfl_xor(psum, 16, 64);
        psum += __shfl_xor(psum, 32, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
#pragma unroll
        for (int d = 0; d < 4; d++) o[d] *= alpha;
        // O^T[d][q] += V^T[d][key] P^T[key][q]; k-step u uses key t*16+4g+i (t=u/4, i=u%4)
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int t = u >> 2, i = u & 3;
                const float a = Vs[(t * 16 + 4 * g + i) * EVS + d * 16 + ql];
                o[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, st[t][i], o[d], 0, 0, 0);
            }
    }
    if (q < N) {
        const float inv = 1.0f / l_run;
        uint16_t *dst = out + (long)(r0 + q) * D + h * 64;
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = f_to_u16(o[d][i] * inv);
    }
}

void launch_enc_attention(const float *qkv, const int *seg_start, const int *seg_len, int n_seg, int max_len, int D, int H,
                          uint16_t *out, hipStream_t s) {
    if (n_seg <= 0 || max_len <= 0) return;
    dim3 grid((max_len + 63) / 64, H, n_seg);
    hipLaunchKernelGGL(enc_attn_kernel, grid, dim3(256), 0, s, qkv, seg_start, seg_len, D, out);
}

// ===================================================== decoder q/k norm + RoPE
// one wave per (row, head); head_dim 128 -> 2 values per lane.  q heads
// first, then k heads; v heads are copied into the cache.
__global__ __launch_bounds__(256) void qkv_post_kernel(QkvPostArgs a) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nh = a.n_head, nkv = a.n_kv_head;
    const int per_row = nh + 2 * nkv;
    if (wave >= a.rows * per_row) return;
    const int row = wave / per_row, hh = wave - row * per_row;
    const int QD = nh * 128, KD = nkv * 128;
    const float *src = a.qkv + (long)row * (QD + 2 * KD);
    const int pos = a.row_pos[row], seq = a.row_seq[row];
    if (hh >= nh + nkv) {   // V: ggml_cpy f32 -> f16 into the cache
        const int g = hh - nh - nkv;
        const float *v = src + QD + KD + g * 128;
        uint16_t *dst = a.vc + (((long)seq * nkv + g) * a.max_ctx + pos) * 128;
        dst[lane] = f_to_u16(v[lane]);
        dst[lane + 64] = f_to_u16(v[lane + 64]);
        return;
    }
    const bool isq = hh < nh;
    const float *x = isq ? src + hh * 128 : src + QD + (hh - nh) * 128;
    const float *w = isq ? a.q_norm : a.k_norm;
    float x0 = x[lane], x1 = x[lane + 64];
    // ggml_rms_norm (sum of squares in double) + ggml_mul
    double ss = (double)(x0 * x0) + (double)(x1 * x1);
    ss = wave_sum_d(ss);
    const float mean = (float)(ss / 128.0);
    const float scale = 1.0f / sqrtf(mean + a.eps);
    x0 = fmul_rn(fmul_rn(x0, scale), w[lane]);
    x1 = fmul_rn(fmul_rn(x1, scale), w[lane + 64]);
    // NEOX rotation: pair (i, i+64), theta from the host table
    const float2 cs = *(const float2 *)(a.rope + ((long)pos * 64 + lane) * 2);
    const float y0 = x0 * cs.x - x1 * cs.y;
    const float y1 = x0 * cs.y + x1 * cs.x;
    if (isq) {
        uint16_t *dst = a.q_out + (long)row * QD + hh * 128;
        dst[lane] = f_to_u16(y0);
        dst[lane + 64] = f_to_u16(y1);
    } else {
        const int g = hh - nh;
        uint16_t *dst = a.kc + (((long)seq * nkv + g) * a.max_ctx + pos) * 128;
        dst[lane] = f_to_u16(y0);
        dst[lane + 64] = f_to_u16(y1);
    }
}

void launch_qkv_post(const QkvPostArgs &a, hipStream_t s) {
    const long waves = (long)a.rows * (a.n_head + 2 * a.n_kv_head);
    if (waves <= 0) return;
    hipLaunchKernelGGL(qkv_post_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, a);
}

// ================================================= decoder prefill (fp16 MFMA)
#define PK_ROW 128     // K tile: [64 keys][128 d] halves, chunk-swizzled 256 B rows
#define PV_ROW 68      // V^T tile: [128 d][64 keys + 4 pad] halves (136 B rows)

__global__ __launch_bounds__(256) void prefill_attn_kernel(PrefillAttnArgs a) {
    __shared__ __attribute__((aligned(16))) uint16_t Ks[64 * PK_ROW];
    __shared__ __attribute__((aligned(16))) uint16_t Vt[128 * PV_ROW];
    const int sq = blockIdx.z, gk = blockIdx.y;
    const int L = a.seq_len[sq];
    const int q0 = blockIdx.x * 32;
    if (q0 >= L) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, ql = lane & 15;
    const int head = gk * 2 + (wid >> 1);
    const int q = q0 + (wid & 1) * 16 + ql;
    const int row0 = a.seq_row0[sq];
    const int QD = a.n_head * 128;
    const long cbase = ((long)a.seq_slot[sq] * a.n_kv_head + gk) * a.max_ctx;
    const uint16_t *kc = a.kc + cbase * 128, *vc = a.vc + cbase * 128;
    // B operand of S^T = K Q^T (k = d): lane holds Q[q][32s + 8g .. +7]
    half8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; s++)
        qf[s] = q < L ? *(const half8 *)(a.q + (long)(row0 + q) * QD + head * 128 + 32 * s + 8 * g) : half8{};
    floatx4 o[8];
#pragma unroll
    for (int d = 0; d < 8; d++) o[d] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.0f;
    const int kend = min(L, q0 + 32);   // causal: keys <= last query of the block
    for (int k0 = 0; k0 < kend; k0 += 64) {
        __syncthreads();
        for (int i = tid; i < 64 * 16; i += 256) {
            const int key = i >> 4, ch = i & 15;
            u32x4 kv = u32x4{0u, 0u, 0u, 0u}, vv = kv;
            if (k0 + key < L) {
                kv = *(const u32x4 *)(kc + (long)(k0 + key) * 128 + ch * 8);
                vv = *(const u32x4 *)(vc + (long)(k0 + key) * 128 + ch * 8);
            }
            *(u32x4 *)(Ks + key * PK_ROW + ((ch ^ (key & 15)) << 3)) = kv;
            const uint16_t *vh = (const uint16_t *)&vv;
#pragma unroll
            for (int e = 0; e < 8; e++) Vt[(ch * 8 + e) * PV_ROW + key] = vh[e];
        }
        __syncthreads();
        floatx4 st[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            st[t] = floatx4{0.f, 0.f, 0.f, 0.f};
            const int key = t * 16 + ql;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const half8 kf = *(const half8 *)(Ks + key * PK_ROW + (((4 * s + g) ^ (key & 15)) << 3));
                st[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[s], st[t], 0, 0, 0);
            }
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int key = k0 + t * 16 + 4 * g + i;
                float v = st[t][i] * a.scale;
                if (key > q || key >= L) v = -INFINITY;
                st[t][i] = v;
                tmax = fmaxf(tmax, v);
            }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = m_new == -INFINITY ? 1.0f : expf(m_run - m_new);
        float psum = 0.0f;
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float p = m_new == -INFINITY ? 0.0f : expf(st[t][i] - m_new);
                st[t][i] = p;
                psum += p;
            }
        psum += __shfl_xor(psum, 16, 64);
        psum += __shfl_xor(psum, 32, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
#pragma unroll
        for (int d = 0; d < 8; d++) o[d] *= alpha;
        // P^T as the B operand: k-step u covers key sub-tiles 2u (j<4) and 2u+1 (j>=4)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            half8 pf;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                pf[j] = (f16)st[2 * u][j];
                pf[4 + j] = (f16)st[2 * u + 1][j];
            }
#pragma unroll
            for (int d = 0; d < 8; d++) {
                const uint16_t *vr = Vt + (d * 16 + ql) * PV_ROW + 32 * u + 4 * g;
                half4 lo = *(const half4 *)vr;
                half4 hi = *(const half4 *)(vr + 16);
                half8 vf = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf, o[d], 0, 0, 0);
            }
        }
    }
    if (q < L) {
        const float inv = l_run > 0.0f ? 1.0f / l_run : 0.0f;
        uint16_t *dst = a.out + (long)(row0 + q) * QD + head * 128;
#pragma unroll
        for (int d = 0; d < 8; d++)
#pragma unroll
            for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = f_to_u16(o[d][i] * inv);
    }
}

void launch_prefill_attention(const PrefillAttnArgs &a, hipStream_t s) {
    if (a.n_seq <= 0 || a.max_len <= 0) return;
    dim3 grid((a.max_len + 31) / 32, a.n_kv_head, a.n_seq);
    hipLaunchKernelGGL(prefill_attn_kernel, grid, dim3(256), 0, s, a);
}

// ================================================== decoder single token
// grid (max_splits, n_kv_head, B); block 256: 16 lanes per key (8 dims each),
// 4 keys per wave instruction, both q heads of the kv group at once.
__global__ __launch_bounds__(256) void decode_attn_split_kernel(DecodeAttnArgs a) {
    __shared__ float sc[2][512];
    __shared__ float red[2][4][2];
    __shared__ float ored[4][2][128];
    const int b = blockIdx.z, gk = blockIdx.y, sp = blockIdx.x;
    const int nkv = a.n_kv[b];
    const int k0 = sp * a.split_len;
    if (k0 >= nkv) return;
    const int k1 = min(nkv, k0 + a.split_len);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int sub = lane >> 4, dl = (lane & 15) * 8;
    const int QD = a.n_head * 128;
    const long cbase = ((long)a.seq_slot[b] * a.n_kv_head + gk) * a.max_ctx;
    const uint16_t *kc = a.kc + cbase * 128, *vc = a.vc + cbase * 128;
    const half8 q0 = *(const half8 *)(a.q + (long)b * QD + (2 * gk) * 128 + dl);
    const half8 q1 = *(const half8 *)(a.q + (long)b * QD + (2 * gk + 1) * 128 + dl);
    // scores
    for (int kb = k0 + wid * 4; kb < k1; kb += 16) {
        const int key = kb + sub;
        float s0 = 0.f, s1 = 0.f;
        if (key < k1) {
            const half8 kv = *(const half8 *)(kc + (long)key * 128 + dl);
#pragma unroll
            for (int e = 0; e < 8; e++) {
                s0 = fmaf((float)kv[e], (float)q0[e], s0);
                s1 = fmaf((float)kv[e], (float)q1[e], s1);
            }
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            s0 += __shfl_xor(s0, o, 64);
            s1 += __shfl_xor(s1, o, 64);
        }
        if ((lane & 15) == 0 && key < k1) {
            sc[0][key - k0] = s0 * a.scale;
            sc[1][key - k0] = s1 * a.scale;
        }
    }
    __syncthreads();
    const int n = k1 - k0;
    float mx0 = -INFINITY, mx1 = -INFINITY;
    for (int i = tid; i < n; i += 256) { mx0 = fmaxf(mx0, sc[0][i]); mx1 = fmaxf(mx1, sc[1][i]); }
    mx0 = wave_max(mx0);
    mx1 = wave_max(mx1);
    if (lane == 0) { red[0][wid][0] = mx0; red[1][wid][0] = mx1; }
    __syncthreads();
    mx0 = fmaxf(fmaxf(red[0][0][0], red[0][1][0]), fmaxf(red[0][2][0], red[0][3][0]));
    mx1 = fmaxf(fmaxf(red[1][0][0], red[1][1][0]), fmaxf(red[1][2][0], red[1][3][0]));
    float l0 = 0.f, l1 = 0.f;
    for (int i = tid; i < n; i += 256) {
        const float p0 = expf(sc[0][i] - mx0), p1 = expf(sc[1][i] - mx1);
        sc[0][i] = p0;
        sc[1][i] = p1;
        l0 += p0;
        l1 += p1;
    }
    l0 = wave_sum(l0);
    l1 = wave_sum(l1);
    if (lane == 0) { red[0][wid][1] = l0; red[1][wid][1] = l1; }
    __syncthreads();
    // P.V: lane owns 8 dims, 4 keys per wave instruction
    float acc0[8], acc1[8];
#pragma unroll
    for (int e = 0; e < 8; e++) { acc0[e] = 0.f; acc1[e] = 0.f; }
    for (int kb = k0 + wid * 4; kb < k1; kb += 16) {
        const int key = kb + sub;
        if (key < k1) {
            const half8 vv = *(const half8 *)(vc + (long)key * 128 + dl);
            const float p0 = sc[0][key - k0], p1 = sc[1][key - k0];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                acc0[e] = fmaf((float)vv[e], p0, acc0[e]);
                acc1[e] = fmaf((float)vv[e], p1, acc1[e]);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
        acc0[e] += __shfl_xor(acc0[e], 16, 64);
        acc0[e] += __shfl_xor(acc0[e], 32, 64);
        acc1[e] += __shfl_xor(acc1[e], 16, 64);
        acc1[e] += __shfl_xor(acc1[e], 32, 64);
    }
    if (sub == 0) {
#pragma unroll
        for (int e = 0; e < 8; e++) { ored[wid][0][dl + e] = acc0[e]; ored[wid][1][dl + e] = acc1[e]; }
    }
    __syncthreads();
    const int hh = tid >> 7, d = tid & 127;
    const float ov = ored[0][hh][d] + ored[1][hh][d] + ored[2][hh][d] + ored[3][hh][d];
    const int head = 2 * gk + hh;
    const long pidx = ((long)b * a.n_head + head) * a.max_splits + sp;
    a.part_o[pidx * 128 + d] = ov;
    if (d == 0) {
        a.part_ml[pidx * 2 + 0] = hh ? mx1 : mx0;
        a.part_ml[pidx * 2 + 1] = red[hh][0][1] + red[hh][1][1] + red[hh][2][1] + red[hh][3][1];
    }
}

// grid (n_head, B), block 128
__global__ __launch_bounds__(128) void decode_attn_combine_kernel(DecodeAttnArgs a) {
    const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
    const int nsp = (a.n_kv[b] + a.split_len - 1) / a.split_len;
    const long base = ((long)b * a.n_head + h) * a.max_splits;
    float M = -INFINITY;
    for (int s = 0; s < nsp; s++) M = fmaxf(M, a.part_ml[(base + s) * 2]);
    float l = 0.f, o = 0.f;
    for (int s = 0; s < nsp; s++) {
        const float w = expf(a.part_ml[(base + s) * 2] - M);
        l += a.part_ml[(base + s) * 2 + 1] * w;
        o += a.part_o[(base + s) * 128 + d] * w;
    }
    a.out[(long)b * a.n_head * 128 + h * 128 + d] = f_to_u16(l > 0.f ? o / l : 0.f);
}

void launch_decode_attention(const DecodeAttnArgs &a, hipStream_t s) {
    if (a.B <= 0) return;
    hipLaunchKernelGGL(decode_attn_split_kernel, dim3(a.max_splits, a.n_kv_head, a.B), dim3(256), 0, s, a);
    hipLaunchKernelGGL(decode_attn_combine_kernel, dim3(a.n_head, a.B), dim3(128), 0, s, a);
}

}  // namespace qasr
