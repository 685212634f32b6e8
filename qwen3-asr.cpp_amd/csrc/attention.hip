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
#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <stdexcept>

#include "dev_common.h"
#include "fx_chain.h"
#include "fx_decode.h"
#include "kernels.h"

namespace qasr {

// ============================================================ encoder (fp32)
#define EKS 66   // K tile row stride (floats): conflict-free A reads
#define EVS 68   // V tile row stride (floats): conflict-free permuted reads

__global__ __launch_bounds__(256) void enc_attn_kernel(const float *__restrict__ qkv, const int *__restrict__ seg_start,
                                                       const int *__restrict__ seg_len, int D, uint16_t *__restrict__ out,
                                                       float *__restrict__ out32) {
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

    // K / V tiles (64 keys x 64 dims fp32) go global -> registers one tile ahead
    // (the next tile's loads are in flight during this tile's MFMAs: a
    // load-then-compute loop paid a memory latency per tile, ~1/3 of the time
    // at a 1.2k-frame clip), then registers -> LDS at the tile start
    float4 kpre[4], vpre[4];
    auto fetch = [&](int kb) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = tid + 256 * j, key = i >> 4, c4 = (i & 15) * 4;
            kpre[j] = vpre[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (kb + key < N) {
                const float *rowp = qkv + (long)(r0 + kb + key) * ld + h * 64 + c4;
                kpre[j] = *(const float4 *)(rowp + D);
                vpre[j] = *(const float4 *)(rowp + 2 * D);
            }
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < N; k0 += 64) {
        __syncthreads();   // the previous tile's readers are done
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = tid + 256 * j, key = i >> 4, c4 = (i & 15) * 4;
            float *kd = Ks + key * EKS + c4;
            *(float2 *)kd = make_float2(kpre[j].x, kpre[j].y);
            *(float2 *)(kd + 2) = make_float2(kpre[j].z, kpre[j].w);
            *(float4 *)(Vs + key * EVS + c4) = vpre[j];
        }
        __syncthreads();
        if (k0 + 64 < N) fetch(k0 + 64);
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
        if (out32) {
            float *dst = out32 + (long)(r0 + q) * D + h * 64;
#pragma unroll
            for (int d = 0; d < 4; d++)
#pragma unroll
                for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = o[d][i] * inv;
        } else {
            uint16_t *dst = out + (long)(r0 + q) * D + h * 64;
#pragma unroll
            for (int d = 0; d < 4; d++)
#pragma unroll
                for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = f_to_u16(o[d][i] * inv);
        }
    }
}

// ---------------------------------------------- encoder, fp16 MFMA, split operands
// The same flash loop on v_mfma_f32_16x16x32_f16 with every fp32 operand split
// into fp16 hi + lo parts (x = hi + lo to ~22 bits): S = Kh.Qh + Kh.Ql + Kl.Qh,
// O += Vh.Ph + Vh.Pl + Vl.Ph (the lo.lo term, ~2^-22 relative, dropped).  The
// products are exact and accumulate in fp32, so the scores and the output keep
// fp32-level error (the reference's F32 mul_mat, src/audio_encoder.cpp:466-486)
// at 3 f16 MFMAs where the fp32 path spends 8 f32 ones of 4x the cycles.
// Q carries the score scale 1/8 and log2(e) (softmax by v_exp_f32); P is split
// from p * 2^12 so its lo part stays a normal fp16 down to p ~ 2^-14 (the scale
// is folded back with 1/l).  Two wave groups of four take alternate 64-key tiles
// of the same 64 queries (two waves per SIMD on a one-block-per-CU grid) and
// merge their (m, l, O) through LDS at the end.  LDS per group: K hi/lo
// row-major [key][dim], V hi/lo transposed [dim][key'] with the keys permuted
// into the MFMA k order of the P fragments (four consecutive keys stay
// consecutive, so each staging thread writes 8-byte runs).
#define EHS 72   // LDS row stride (halves) of the hi/lo tiles
#define EH_GRP (4 * 64 * EHS)   // halves of one wave group's tiles

__device__ __forceinline__ int eh_vpos(int key) {
    // P.V k-step u takes S^T sub-tiles 2u, 2u+1; lane group g holds keys
    // t*16 + 4g + i -> k index u*32 + 8g + 4*(t&1) + i
    const int t = key >> 4, g = (key >> 2) & 3, i = key & 3;
    return (t >> 1) * 32 + 8 * g + 4 * (t & 1) + i;
}

__global__ __launch_bounds__(512) void enc_attn_h_kernel(const float *__restrict__ qkv, const int *__restrict__ seg_start,
                                                         const int *__restrict__ seg_len, int D, uint16_t *__restrict__ out,
                                                         float *__restrict__ out32) {
    __shared__ __attribute__((aligned(16))) f16 lds[2 * EH_GRP];
    const int b = blockIdx.z, h = blockIdx.y;
    const int N = seg_len[b], r0 = seg_start[b];
    const int qblk = blockIdx.x * 64;
    if (qblk >= N) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int grp = wid >> 2, gtid = tid & 255;
    const int g = lane >> 4, ql = lane & 15;
    f16 *Kh = lds + grp * EH_GRP, *Kl = Kh + 64 * EHS, *Vh = Kh + 2 * 64 * EHS, *Vl = Kh + 3 * 64 * EHS;
    const int ld = 3 * D;
    const int q = qblk + (wid & 3) * 16 + ql;
    const float qscale = 0.125f * 1.4426950408889634f;
    // B operand of S^T = K Q^T, k-step s: lane holds Q[q][32s + 8g + j] * qscale
    half8 qh[2], qlo[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
        if (q < N) {
            const float *qp = qkv + (long)(r0 + q) * ld + h * 64 + 32 * s + 8 * g;
            a = *(const float4 *)qp;
            c = *(const float4 *)(qp + 4);
        }
        const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float x = v[j] * qscale;
            const f16 hi = (f16)x;
            qh[s][j] = hi;
            qlo[s][j] = (f16)(x - (float)hi);
        }
    }
    floatx4 o[4];
#pragma unroll
    for (int d = 0; d < 4; d++) o[d] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.0f;

    // staging thread: keys 4*kq .. 4*kq+3 of the tile, dims c4 .. c4+3
    const int kq = gtid >> 4, c4 = (gtid & 15) * 4;
    float4 kpre[4], vpre[4];
    auto fetch = [&](int kb) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int key = kb + 4 * kq + r;
            kpre[r] = vpre[r] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (key < N) {
                const float *rowp = qkv + (long)(r0 + key) * ld + h * 64 + c4;
                kpre[r] = *(const float4 *)(rowp + D);
                vpre[r] = *(const float4 *)(rowp + 2 * D);
            }
        }
    };
    const int ntile = (N + 63) >> 6;
    const int niter = (ntile + 1) >> 1;
    if (grp < ntile) fetch(grp * 64);
    for (int it = 0; it < niter; it++) {
        const int tile = 2 * it + grp;
        const bool live = tile < ntile;   // the odd group's last tile may not exist
        const int k0 = tile * 64;
        __syncthreads();   // the previous tile's readers are done
        if (live) {
            const int vp = eh_vpos(4 * kq);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float kv[4] = {kpre[r].x, kpre[r].y, kpre[r].z, kpre[r].w};
                half4 kh, kl;
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const f16 hk = (f16)kv[e];
                    kh[e] = hk;
                    kl[e] = (f16)(kv[e] - (float)hk);
                }
                *(half4 *)(Kh + (4 * kq + r) * EHS + c4) = kh;
                *(half4 *)(Kl + (4 * kq + r) * EHS + c4) = kl;
            }
            const float vv[4][4] = {{vpre[0].x, vpre[0].y, vpre[0].z, vpre[0].w},
                                    {vpre[1].x, vpre[1].y, vpre[1].z, vpre[1].w},
                                    {vpre[2].x, vpre[2].y, vpre[2].z, vpre[2].w},
                                    {vpre[3].x, vpre[3].y, vpre[3].z, vpre[3].w}};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                half4 vh, vl;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const f16 hv = (f16)vv[r][e];
                    vh[r] = hv;
                    vl[r] = (f16)(vv[r][e] - (float)hv);
                }
                *(half4 *)(Vh + (c4 + e) * EHS + vp) = vh;
                *(half4 *)(Vl + (c4 + e) * EHS + vp) = vl;
            }
        }
        __syncthreads();
        if (!live) continue;
        if (tile + 2 < ntile) fetch(k0 + 128);
        floatx4 st[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            st[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int off = (t * 16 + ql) * EHS + 32 * s + 8 * g;
                const half8 ah = *(const half8 *)(Kh + off), al = *(const half8 *)(Kl + off);
                st[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, qh[s], st[t], 0, 0, 0);
                st[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, qlo[s], st[t], 0, 0, 0);
                st[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, qh[s], st[t], 0, 0, 0);
            }
        }
        // lane holds the scaled (log2-domain) S[q][key = k0 + t*16 + 4g + i]
        if (k0 + 64 > N) {
#pragma unroll
            for (int t = 0; t < 4; t++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (k0 + t * 16 + 4 * g + i >= N) st[t][i] = -INFINITY;
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) tmax = fmaxf(tmax, st[t][i]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        float psum = 0.0f;
        half8 ph[2], pl[2];
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float p = __builtin_amdgcn_exp2f(st[t][i] - m_new);
                psum += p;
                const float ps = p * 4096.0f;
                const f16 hi = (f16)ps;
                ph[t >> 1][4 * (t & 1) + i] = hi;
                pl[t >> 1][4 * (t & 1) + i] = (f16)(ps - (float)hi);
            }
        psum += __shfl_xor(psum, 16, 64);
        psum += __shfl_xor(psum, 32, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
#pragma unroll
        for (int d = 0; d < 4; d++) o[d] *= alpha;
        // O^T[d][q] += V^T[d][key'] P^T[key'][q]
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int off = (d * 16 + ql) * EHS + 32 * u + 8 * g;
                const half8 ah = *(const half8 *)(Vh + off), al = *(const half8 *)(Vl + off);
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, ph[u], o[d], 0, 0, 0);
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, pl[u], o[d], 0, 0, 0);
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, ph[u], o[d], 0, 0, 0);
            }
    }
    // merge the two groups: group 1 parks (m, l, O) in LDS, group 0 combines
    __syncthreads();
    float *park = (float *)lds;   // [4 waves][18][64 lanes]
    if (grp == 1) {
        float *pw = park + (wid & 3) * 18 * 64 + lane;
        pw[0] = m_run;
        pw[64] = l_run;
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int i = 0; i < 4; i++) pw[(2 + 4 * d + i) * 64] = o[d][i];
    }
    __syncthreads();
    if (grp == 1 || q >= N) return;
    {
        const float *pw = park + (wid & 3) * 18 * 64 + lane;
        const float m1 = pw[0], l1 = pw[64];
        const float m = fmaxf(m_run, m1);
        const float a0 = __builtin_amdgcn_exp2f(m_run - m), a1 = __builtin_amdgcn_exp2f(m1 - m);
        l_run = l_run * a0 + l1 * a1;
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int i = 0; i < 4; i++) o[d][i] = o[d][i] * a0 + pw[(2 + 4 * d + i) * 64] * a1;
    }
    const float inv = (1.0f / l_run) * (1.0f / 4096.0f);
    if (out32) {
        float *dst = out32 + (long)(r0 + q) * D + h * 64;
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = o[d][i] * inv;
    } else {
        uint16_t *dst = out + (long)(r0 + q) * D + h * 64;
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = f_to_u16(o[d][i] * inv);
    }
}

void launch_enc_attention(const float *qkv, const int *seg_start, const int *seg_len, int n_seg, int max_len, int D, int H,
                          uint16_t *out, hipStream_t s, float *out32, bool f32_mfma) {
    if (n_seg <= 0 || max_len <= 0) return;
    if (D != H * 64) throw std::runtime_error("encoder attention: head_dim must be 64");
    dim3 grid((max_len + 63) / 64, H, n_seg);
    if (f32_mfma)
        hipLaunchKernelGGL(enc_attn_kernel, grid, dim3(256), 0, s, qkv, seg_start, seg_len, D, out, out32);
    else
        hipLaunchKernelGGL(enc_attn_h_kernel, grid, dim3(512), 0, s, qkv, seg_start, seg_len, D, out, out32);
}

// ===================================================== decoder q/k norm + RoPE
// one wave per (row, HPW consecutive heads of one kind), head_dim 128 -> 2
// values per lane per head.  q heads first, then k heads; v heads are copied
// into the caches.  All HPW heads' loads are issued before any use: with one
// head a wave (2 x 256 B in flight) the launch ran at the wave-slot bound of
// bytes in flight (~2.3 TB/s at 64 x 405 rows); 4 heads a wave quadruple it.
template <int HPW>
__global__ __launch_bounds__(256) void qkv_post_kernel(QkvPostArgs a) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nh = a.n_head, nkv = a.n_kv_head;
    const int per_row = (nh + 2 * nkv) / HPW;
    if (wave >= a.rows * per_row) return;
    const int row = wave / per_row, hh0 = (wave - row * per_row) * HPW;
    const int QD = nh * 128, KD = nkv * 128;
    const float *src = a.qkv + (long)row * (QD + 2 * KD);
    const int pos = a.row_pos[row], seq = a.row_seq[row];
    float x0[HPW], x1[HPW];
#pragma unroll
    for (int u = 0; u < HPW; u++) {   // the q / k / v column blocks are contiguous: head hh at src + 128 hh
        x0[u] = src[(hh0 + u) * 128 + lane];
        x1[u] = src[(hh0 + u) * 128 + lane + 64];
    }
    if (hh0 >= nh + nkv) {   // V: ggml_cpy f32 -> f16 into the cache
#pragma unroll
        for (int u = 0; u < HPW; u++) {
            const int g = hh0 + u - nh - nkv;
            uint16_t *dst = a.vc + (((long)seq * nkv + g) * a.max_ctx + pos) * 128;
            const uint16_t v0 = f_to_u16(x0[u]), v1 = f_to_u16(x1[u]);
            dst[lane] = v0;
            dst[lane + 64] = v1;
            uint16_t *t = a.vt + ((long)seq * nkv + g) * 128 * vt_ctx(a.max_ctx);
            t[vt_index(pos, lane)] = v0;
            t[vt_index(pos, lane + 64)] = v1;
        }
        return;
    }
    const bool isq = hh0 < nh;
    const float *w = isq ? a.q_norm : a.k_norm;
    const float w0 = w[lane], w1 = w[lane + 64];
    const float2 cs = *(const float2 *)(a.rope + ((long)pos * 64 + lane) * 2);
#pragma unroll
    for (int u = 0; u < HPW; u++) {
        const int hh = hh0 + u;
        // ggml_rms_norm (sum of squares in double) + ggml_mul
        double ss = (double)(x0[u] * x0[u]) + (double)(x1[u] * x1[u]);
        ss = wave_sum_d(ss);
        const float mean = (float)(ss / 128.0);
        const float scale = 1.0f / sqrtf(mean + a.eps);
        const float n0 = fmul_rn(fmul_rn(x0[u], scale), w0);
        const float n1 = fmul_rn(fmul_rn(x1[u], scale), w1);
        // NEOX rotation: pair (i, i+64), theta from the host table
        const float y0 = n0 * cs.x - n1 * cs.y;
        const float y1 = n0 * cs.y + n1 * cs.x;
        if (a.q32) {   // fp32 copies (ForcedAligner: ggml_flash_attn_ext on fp32 Q and K)
            float *d32 = isq ? a.q32 + (long)row * QD + hh * 128 : a.k32 + (long)row * KD + (hh - nh) * 128;
            d32[lane] = y0;
            d32[lane + 64] = y1;
        }
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
}

void launch_qkv_post(const QkvPostArgs &a, hipStream_t s) {
    const int heads = a.n_head + 2 * a.n_kv_head;
    const long waves1 = (long)a.rows * heads;
    if (waves1 <= 0) return;
    if (a.n_head % 4 == 0 && a.n_kv_head % 4 == 0) {
        const long waves = waves1 / 4;
        hipLaunchKernelGGL(qkv_post_kernel<4>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(qkv_post_kernel<1>, dim3((unsigned)((waves1 + 3) / 4)), dim3(256), 0, s, a);
    }
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
    const int P0 = a.seq_pos0 ? a.seq_pos0[sq] : 0;   // a chunk after P0 cached tokens: query t at position P0 + t
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, ql = lane & 15;
    const int head = gk * 2 + (wid >> 1);
    const int q = q0 + (wid & 1) * 16 + ql;
    const int qp = P0 + q, KL = P0 + L;   // the query's position; keys 0 .. KL - 1
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
    const int kend = min(KL, P0 + q0 + 32);   // causal: keys <= last query of the block
    for (int k0 = 0; k0 < kend; k0 += 64) {
        __syncthreads();
        for (int i = tid; i < 64 * 16; i += 256) {
            const int key = i >> 4, ch = i & 15;
            u32x4 kv = u32x4{0u, 0u, 0u, 0u}, vv = kv;
            if (k0 + key < KL) {
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
                if (key > qp || key >= KL) v = -INFINITY;
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
        // P^T as the B operand: k-step u covers key sub-tiles 2u (j<4) and 2u+1 (j>=4).
        // P is fp32 in ggml's FA; it enters the f16 MFMA as hi + lo fp16 parts
        // (p = hi + lo to ~2^-22), so P.V keeps fp32-accurate weights.
#pragma unroll
        for (int u = 0; u < 2; u++) {
            half8 pf, pl;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                pf[j] = (f16)st[2 * u][j];
                pf[4 + j] = (f16)st[2 * u + 1][j];
                pl[j] = (f16)(st[2 * u][j] - (float)pf[j]);
                pl[4 + j] = (f16)(st[2 * u + 1][j] - (float)pf[4 + j]);
            }
#pragma unroll
            for (int d = 0; d < 8; d++) {
                const uint16_t *vr = Vt + (d * 16 + ql) * PV_ROW + 32 * u + 4 * g;
                half4 lo = *(const half4 *)vr;
                half4 hi = *(const half4 *)(vr + 16);
                half8 vf = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf, o[d], 0, 0, 0);
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pl, o[d], 0, 0, 0);
            }
        }
    }
    if (q < L) {
        const float inv = l_run > 0.0f ? 1.0f / l_run : 0.0f;
        if (a.out32) {
            float *dst = a.out32 + (long)(row0 + q) * QD + head * 128;
#pragma unroll
            for (int d = 0; d < 8; d++)
#pragma unroll
                for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = o[d][i] * inv;
        } else {
            uint16_t *dst = a.out + (long)(row0 + q) * QD + head * 128;
#pragma unroll
            for (int d = 0; d < 8; d++)
#pragma unroll
                for (int i = 0; i < 4; i++) dst[d * 16 + 4 * g + i] = f_to_u16(o[d][i] * inv);
        }
    }
}

void launch_prefill_attention(const PrefillAttnArgs &a, hipStream_t s) {
    if (a.n_seq <= 0 || a.max_len <= 0) return;
    dim3 grid((a.max_len + 31) / 32, a.n_kv_head, a.n_seq);
    hipLaunchKernelGGL(prefill_attn_kernel, grid, dim3(256), 0, s, a);
}

// ================================================== decoder single token
// grid (grid_splits, n_kv_head, B), block 256 (4 waves).  Split = 64 keys, so a
// 1.5k-token context spreads over ~190 workgroups (one CU streams only ~32 KB).
// Every K/V row of the split -- and the raw q/k/v of the token -- is requested
// at kernel entry, before the device-resident position is known: the split
// costs about one HBM latency.  Each block normalises + rotates the two q heads
// of its kv group (src/text_decoder.cpp:640-700: rms_norm, NEOX RoPE); the
// block owning the last split also builds the new key, writes K/V into the fp16
// cache and uses them from LDS.  Partials (unnormalised O, max, sum) are
// published write-through (sc1 16-B stores, drained) and counted with one
// agent-scope atomic per block; the last arriver of the kv group reads them back
// with sc1 loads, combines (S_inv = 1/S as ggml's flash_attn_ext) and writes the
// fp16 attention output (MI355X_MICROARCH.md, inter-workgroup hand-off table,
// row 1).  Counters are zero at rest: the last arriver re-arms its own.
#define DSPLIT 64   // split of the batch-1..8 grid; larger batches use 256-key splits
#define DWAVES 4

__device__ __forceinline__ void st_sc1_x4(float *p, float4 f) {
    const floatx4 v = {f.x, f.y, f.z, f.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// nine 16-B sc1 loads (element tid + 256 j of src, clamped to n4 - 1) issued
// back to back and drained in the same asm block, so no copy of an output can
// be scheduled before the data has landed
__device__ __forceinline__ void ld_sc1_x4_burst5(const floatx4 *src, int tid, int n4, floatx4 *v) {
    const floatx4 *p[5];
#pragma unroll
    for (int j = 0; j < 5; j++) p[j] = src + min(tid + 256 * j, n4 - 1);
    asm volatile(
        "global_load_dwordx4 %0, %5, off sc1\n\t"
        "global_load_dwordx4 %1, %6, off sc1\n\t"
        "global_load_dwordx4 %2, %7, off sc1\n\t"
        "global_load_dwordx4 %3, %8, off sc1\n\t"
        "global_load_dwordx4 %4, %9, off sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4])
        : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4])
        : "memory");
}
// four 16-B sc1 loads (p, p + 512 halves, p + 1024, p + 1536) drained in the same asm block
__device__ __forceinline__ void ld_sc1_x4_4(const uint16_t *p, u32x4 *v) {
    asm volatile(
        "global_load_dwordx4 %0, %4, off sc1\n\t"
        "global_load_dwordx4 %1, %4, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %4, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %4, off offset:3072 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
        : "v"(p)
        : "memory");
}

// a K/V cache row piece: read once per step by one CU -- nontemporal when
// DecodeAttnArgs.kv_nt (MI355X_MICROARCH.md nt-weights), else default policy
__device__ __forceinline__ half8 kv_load(const uint16_t *p, int nt) {
    return nt ? __builtin_nontemporal_load((const half8 *)p) : *(const half8 *)p;
}

// a split workgroup's LDS (decode_attn_body): its own __shared__ object in the
// split kernel, one layout of the fused launch's shared role buffer there
template <int SPL>
struct alignas(16) SplitLds {
    uint16_t qs[2][128];
    uint16_t knew[128];
    uint16_t vnew[128];
    float sc[2][SPL];
    float ored[DWAVES * 4][2][128];   // [wave x row][head][dim]
    float cml[2][2];
    int last;
};
template <int SPL, bool FUSED>
__device__ __forceinline__ void decode_attn_body(const DecodeAttnArgs a, const int sp, const int g, const int b, const int nsp,
                                                 SplitLds<SPL> &SL) {
    auto &qs = SL.qs;
    auto &knew = SL.knew;
    auto &vnew = SL.vnew;
    auto &sc = SL.sc;
    auto &ored = SL.ored;
    auto &cml = SL.cml;
    auto &last = SL.last;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int QD = a.n_head * 128, KD = a.n_kv_head * 128;
    const long blk = sp + (long)nsp * (g + (long)a.n_kv_head * b);   // dev-trace row
    auto mark = [&](int slot) {
        if (a.trace && tid == 0) a.trace[blk * 8 + slot] = rt_now();
    };
    mark(0);
    // ---- the token's raw vectors, one per wave: wave 0/1 = q heads 2g/2g+1,
    //      wave 2 = k, wave 3 = v of group g; lane owns dims lane and lane + 64
    //      (the NEOX RoPE pair), so norm and rotation need no LDS round trip
    const float *raw = a.qkv + (long)b * (QD + 2 * KD);
    const float *src = wid < 2 ? raw + (2 * g + wid) * 128 : raw + QD + (wid - 2) * KD + g * 128;
    float x0 = 0.f, x1 = 0.f;
    if constexpr (!FUSED) { x0 = src[lane]; x1 = src[lane + 64]; }
    const float *nw = wid < 2 ? a.q_norm : a.k_norm;
    const float w0 = nw[lane], w1 = nw[lane + 64];
    if constexpr (FUSED)   // let the QKV blocks' weight stream get ahead in the memory queues
        for (int i = 0; i < a.fuse_delay; i++) __builtin_amdgcn_s_sleep(8);
    // ---- every K/V row of the split (addresses depend on blockIdx only).  Decode
    //      rows are cache slots: row b of a decode step is slot b (qasr_run_stream
    //      refills a finished slot in place, its prefill writing through seq_slot
    //      = b), so b indexes the K/V and V^T caches alike.  Rows past the position
    //      are masked below; the cache is zero-initialised so they are finite.
    const long cbase = ((long)b * a.n_kv_head + g) * a.max_ctx;
    uint16_t *kc = a.kc + cbase * 128, *vc = a.vc + cbase * 128;
    const int k0 = sp * SPL;
    const int sub = lane >> 4, dl = (lane & 15) * 8;
    const int q4 = lane >> 4, c16 = lane & 15;
    constexpr int KPW = SPL / DWAVES / 4;   // V rows per lane (4 or 16)
    constexpr int TW = SPL / DWAVES / 16;   // 16-key MFMA tiles per wave (1 or 4)
    // separate launches (decode batches, long kernels): keys past this
    // sequence's position re-read its last row -- cache hits instead of HBM
    // traffic for the masked tail of a short sequence in a batch whose grid
    // covers the longest; the fused batch-1 launch keeps its K/V requests free
    // of the dependent position load (see below)
    const int kcap = FUSED ? a.max_ctx - 1 : min(a.pos[b], a.max_ctx - 1);
    // K in the v_mfma_f32_16x16x32_f16 B layout: tile t, step s -> key 16t + c16
    // of this wave's range, dims 32s + 8q4 .. +8 (16 rows x 64 B per load)
    half8 kk[TW][4], vv[KPW];
#pragma unroll
    for (int t = 0; t < TW; t++)
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            const int key = min(k0 + wid * (SPL / DWAVES) + 16 * t + c16, kcap);
            kk[t][s4] = kv_load(kc + (long)key * 128 + 32 * s4 + 8 * q4, a.kv_nt);
        }
    if (FUSED && a.fx) {   // exact attention: no V here; this split's keys' V^T rows -> this XCD's L2 for the chain
        if (a.fx_vpf & 1) {
            const uint16_t *vt = a.vt + ((long)b * a.n_kv_head + g) * 128 * vt_ctx(a.max_ctx) + (long)(k0 / 8) * 1024;
#pragma unroll
            for (int i = 0; i < KPW; i++) vv[i] = *(const half8 *)(vt + (long)(i * 256 + tid) * 8);
        }
    } else if (!a.scores) {   // scores mode reads no V
#pragma unroll
        for (int i = 0; i < KPW; i++) {
            const int key = min(k0 + wid * (SPL / DWAVES) + i * 4 + sub, kcap);
            vv[i] = kv_load(vc + (long)key * 128 + dl, a.kv_nt);
        }
    }
    // No exit test on the position anywhere: with one, hipcc hoists the
    // dependent pos load and the test in front of the K/V requests (two memory
    // latencies in series).  The host sizes the grid to the context
    // (grid_splits, a 256-key bucket); a split past this sequence's end is
    // fully masked and publishes an empty partial (m = -inf, l = 0, O = 0).
    if (FUSED && a.gran) {
        // granule hand-off: each lane polls its own two {value, tag} granules
        // (sc1 loads) until both carry this step's tag -- the data arrives with
        // its own flag, no drain / arrival count / second load (MI355X guide,
        // hand-off table: data-tagged granules).  Bounded like the counter wait.
        const uint32_t tag = gran_tag(a.pos[b], a.layer);
        const unsigned long long *gp = a.gran + (src - raw) + lane;
        unsigned long long v0 = 0, v1 = 0;
        bool ok = false;
        for (int it = 0; it < a.poll_limit; it++) {
            v0 = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v1 = __hip_atomic_load(gp + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(v0 >> 32) == tag && (uint32_t)(v1 >> 32) == tag;
            if (__all(ok)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!__all(ok) && lane == 0) __hip_atomic_fetch_or(a.err, (unsigned)DEVERR_QKV_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x0 = __uint_as_float((uint32_t)v0);
        x1 = __uint_as_float((uint32_t)v1);
    } else if constexpr (FUSED) {
        // wait for the kv group's 64 QKV workgroups (bounded: a lost arrival must
        // not hang the GPU), then read their write-through outputs with sc1 loads
        // A wait that runs out sets DEVERR_QKV_WAIT and the split still
        // publishes (its partial is then garbage, the call returns an error):
        // skipping it would only strand the combiner and the o-proj blocks.
        if (tid == 0) {
            int ok = 0;
            for (int it = 0; it < a.poll_limit; it++) {
                // replica sp % 8 of the group's counter (8 replicas, one 64-B line each):
                // the pollers of a group spread over 8 lines instead of one hot word
                if (__hip_atomic_load(a.qcnt + (g * 8 + (sp & 7)) * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                    (a.qkv_need ? a.qkv_need : 64u)) {
                    ok = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            if (a.fence) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (!ok) __hip_atomic_fetch_or(a.err, (unsigned)DEVERR_QKV_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        const uint32_t *sr = (const uint32_t *)src;
        x0 = __uint_as_float(__hip_atomic_load(sr + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        x1 = __uint_as_float(__hip_atomic_load(sr + lane + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    const int pos = a.pos[b];
    const int nkv = pos + 1;
    const int k1 = min(nkv, k0 + SPL);
    const bool lastsp = sp == (nkv - 1) / SPL;
    const float2 cs = *(const float2 *)(a.rope + ((long)pos * 64 + lane) * 2);
    // ---- ggml_rms_norm (double sum of fp32 squares) * weight, NEOX RoPE
    //      (src/text_decoder.cpp:640-700); v is only cast to fp16
    if (wid < 3) {
        const double ss = wave_sum_d((double)(x0 * x0) + (double)(x1 * x1));
        const float scale = 1.0f / sqrtf((float)(ss / 128.0) + a.eps);
        const float y0 = fmul_rn(fmul_rn(x0, scale), w0), y1 = fmul_rn(fmul_rn(x1, scale), w1);
        const uint16_t r0 = f_to_u16(y0 * cs.x - y1 * cs.y), r1 = f_to_u16(y0 * cs.y + y1 * cs.x);
        if (wid < 2) {
            qs[wid][lane] = r0;
            qs[wid][lane + 64] = r1;
        } else if (lastsp) {
            knew[lane] = r0; knew[lane + 64] = r1;
            kc[(long)pos * 128 + lane] = r0;
            kc[(long)pos * 128 + lane + 64] = r1;
        }
    } else if (lastsp) {
        const uint16_t v0 = f_to_u16(x0), v1 = f_to_u16(x1);   // ggml_cpy f32 -> f16
        vnew[lane] = v0; vnew[lane + 64] = v1;
        vc[(long)pos * 128 + lane] = v0;
        vc[(long)pos * 128 + lane + 64] = v1;
        uint16_t *t = a.vt + ((long)b * a.n_kv_head + g) * 128 * vt_ctx(a.max_ctx);
        t[vt_index(pos, lane)] = v0;
        t[vt_index(pos, lane + 64)] = v1;
    }
    __syncthreads();
    // ---- scores S = Q K^T on MFMA: A = the two q heads (rows 0, 1; rows 2-15
    //      zero), B = K^T; lane (q4 = 0, c16) gets S[head r][key c16] in acc[r].
    //      Exact fp16 x fp16 products summed in fp32 (ggml FA: Q cast to fp16).
    if (a.trace) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); mark(1); }
    half8 qa[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; s4++)
        qa[s4] = c16 < 2 ? *(const half8 *)&qs[c16][32 * s4 + 8 * q4] : half8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < TW; t++) {
        const int j = wid * (SPL / DWAVES) + 16 * t + c16;
        if (k0 + j == pos)
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++) kk[t][s4] = *(const half8 *)&knew[32 * s4 + 8 * q4];
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(qa[s4], kk[t][s4], acc, 0, 0, 0);
        if (q4 == 0) {
            const bool ok = k0 + j < k1;
            sc[0][j] = ok ? acc[0] * a.scale : -INFINITY;
            sc[1][j] = ok ? acc[1] * a.scale : -INFINITY;
        }
    }
#pragma unroll
    for (int i = 0; i < KPW; i++) {
        const int j = wid * (SPL / DWAVES) + i * 4 + sub;
        if (k0 + j == pos) vv[i] = *(const half8 *)&vnew[dl];
    }
    __syncthreads();
    mark(6);
    if constexpr (FUSED) {
        if (a.fx) {   // exact attention: the scaled scores to the kv group's chain workgroup, one {fp32, tag} granule each
            const uint32_t tag = gran_tag(pos, a.layer);
            if (tid < 2 * SPL) {
                const int hh = tid / SPL, j = tid - hh * SPL;
                if (k0 + j < k1)
                    __hip_atomic_store(a.sgran + (long)(2 * g + hh) * sgran_ld(a.max_ctx) + k0 + j,
                                       ((unsigned long long)tag << 32) | __float_as_uint(sc[hh][j]), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            if (a.fx_vpf & 1)
#pragma unroll
                for (int i = 0; i < KPW; i++) asm volatile("" ::"v"(vv[i]));   // (the V^T pull has landed)
            mark(3);
            return;
        }
    }
    if constexpr (!FUSED) {
        if (a.scores) {   // front half of the exact attention (fa_exact.hip): this split's scaled scores
            float *dst = a.scores + ((long)b * a.n_head + 2 * g) * a.max_ctx + k0;
            for (int i = tid; i < 2 * SPL; i += 256) {
                const int hh = i / SPL, j = i - hh * SPL;
                if (k0 + j < k1) dst[(long)hh * a.max_ctx + j] = sc[hh][j];
            }
            return;
        }
    }
    // ---- split-local softmax statistics: wave h owns head h, lane = key (mod 64)
    if (wid < 2) {
        constexpr int KL = SPL / 64;
        float v[KL], mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < KL; i++) { v[i] = sc[wid][lane + 64 * i]; mx = fmaxf(mx, v[i]); }
        const float M = wave_max(mx);
        float ps = 0.f;
#pragma unroll
        for (int i = 0; i < KL; i++) {
            const float p = k0 + lane + 64 * i < k1 ? expf(v[i] - M) : 0.f;
            sc[wid][lane + 64 * i] = p;
            ps += p;
        }
        const float l = wave_sum(ps);
        if (lane == 0) { cml[wid][0] = M; cml[wid][1] = l; }
    }
    __syncthreads();
    mark(7);
    // ---- P.V in fp32 (probabilities kept fp32: a Q8_0 o-proj re-quantises
    //      this output, so its rounding must not move)
    float acc0[8], acc1[8];
#pragma unroll
    for (int e = 0; e < 8; e++) { acc0[e] = 0.f; acc1[e] = 0.f; }
#pragma unroll
    for (int i = 0; i < KPW; i++) {
        const int j = wid * (SPL / DWAVES) + i * 4 + sub;
        const float p0 = sc[0][j], p1 = sc[1][j];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const float v = (float)vv[i][e];
            acc0[e] = fmaf(v, p0, acc0[e]);
            acc1[e] = fmaf(v, p1, acc1[e]);
        }
    }
    // per-(wave, row) partial sums go to LDS; the 16-way sum happens once, below
    *(floatx4 *)&ored[wid * 4 + sub][0][dl] = floatx4{acc0[0], acc0[1], acc0[2], acc0[3]};
    *(floatx4 *)&ored[wid * 4 + sub][0][dl + 4] = floatx4{acc0[4], acc0[5], acc0[6], acc0[7]};
    *(floatx4 *)&ored[wid * 4 + sub][1][dl] = floatx4{acc1[0], acc1[1], acc1[2], acc1[3]};
    *(floatx4 *)&ored[wid * 4 + sub][1][dl + 4] = floatx4{acc1[4], acc1[5], acc1[6], acc1[7]};
    __syncthreads();
    mark(2);
    // ---- publish this split's partial: [2 heads][O 128 | m, l, 0, 0], 16-B sc1 stores
    float *gpart = a.part + (((long)b * a.n_kv_head + g) * a.max_splits) * 2 * 132;
    if (tid < 66) {
        const int h = tid / 33, q = tid - h * 33;
        float4 v;
        if (q < 32) {
            floatx4 t = *(const floatx4 *)&ored[0][h][4 * q];
#pragma unroll
            for (int w = 1; w < DWAVES * 4; w++) t += *(const floatx4 *)&ored[w][h][4 * q];
            v = make_float4(t[0], t[1], t[2], t[3]);
        } else {
            v = make_float4(cml[h][0], cml[h][1], 0.f, 0.f);
        }
        st_sc1_x4(gpart + ((long)sp * 2 + h) * 132 + 4 * q, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned int *cnt = a.counter + (long)b * a.n_kv_head + g;
    if (tid == 0) last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nsp - 1;
    __syncthreads();
    mark(3);
    if (!last) return;
    // ---- last arriver: combine the partials of both heads (empty ones weigh 0).
    //      Thread (head hh, dim d) loads its dimension and the (m, l) pair of up
    //      to 16 splits at a time with sc1 loads (all in flight together, one
    //      memory latency per pass) and merges them in registers with the usual
    //      online rescale: no LDS staging, no barrier.
    if (tid == 0) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (FUSED)   // every split is past its wait: re-arm the 8 replicas
            for (int r = 0; r < 8; r++) __hip_atomic_store(a.qcnt + (g * 8 + r) * 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int hh = tid >> 7, d = tid & 127;
    float M = -INFINITY, L = 0.f, O = 0.f;
    for (int s0 = 0; s0 < nsp; s0 += 16) {
        const int ns = min(16, nsp - s0);
        float ov[16];
        unsigned long long ml[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const float *pp = gpart + ((long)(s0 + min(u, ns - 1)) * 2 + hh) * 132;
            ov[u] = __uint_as_float(__hip_atomic_load((const uint32_t *)(pp + d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            ml[u] = __hip_atomic_load((const unsigned long long *)(pp + 128), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (s0 == 0) mark(5);
        float Mn = M;
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (u < ns) Mn = fmaxf(Mn, __uint_as_float((uint32_t)ml[u]));
        const float r = expf(M - Mn);   // first pass: exp(-inf) = 0 on L = O = 0
        float lp = 0.f, op = 0.f;
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (u < ns) {
                const float w = __expf(__uint_as_float((uint32_t)ml[u]) - Mn);
                lp = fadd_rn(lp, fmul_rn(__uint_as_float((uint32_t)(ml[u] >> 32)), w));
                op = fmaf(w, ov[u], op);
            }
        L = L * r + lp;
        O = O * r + op;
        M = Mn;
    }
    const float inv = L > 0.f ? 1.0f / L : 0.f;   // ggml: S_inv = 1/S, VKQ *= S_inv
    if (a.outq) {   // quantised for the Q8_0 o-proj: a 32-block = 32 lanes of one wave
        const float v = O * inv;
        float am = fabsf(v);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
        const long e = (long)b * QD + (2 * g + hh) * 128 + d;
        a.outq[e] = q8_quant(v, am);
        if ((d & 31) == 0) a.outd[e >> 5] = q8_scale(am);
    } else if (a.out32) a.out32[(long)b * QD + (2 * g + hh) * 128 + d] = O * inv;
    else if (FUSED && a.att_done) {
        // the o-proj blocks of this launch read it: write-through 4-byte pairs,
        // every wave drained, then one arrival per replica of att_done
        const uint32_t h = f_to_u16(O * inv);
        const uint32_t hn = __shfl_xor(h, 1, 64);
        if ((d & 1) == 0)
            __hip_atomic_store((uint32_t *)(a.out + (long)b * QD + (2 * g + hh) * 128 + d), h | (hn << 16), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (a.fence && tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (a.fence) __syncthreads();
        if (tid < 8) __hip_atomic_fetch_add(a.att_done + tid * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else a.out[(long)b * QD + (2 * g + hh) * 128 + d] = f_to_u16(O * inv);
    mark(4);
}

template <int SPL>
__global__ __launch_bounds__(256) void decode_attn_kernel(DecodeAttnArgs a) {
    stamp_start(a.stamp);
    __shared__ SplitLds<SPL> SL;
    decode_attn_body<SPL, false>(a, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, SL);
    stamp_end(a.stamp);
}

// ------------------------------------------ decode batches: one workgroup per sequence
// decode_attn_kernel<256> needs 168 VGPRs (a whole split's K/V in flight in
// registers), so 2 workgroups fit a CU: a batch-64 grid of 1024 splits ran in
// two rounds with HBM idle through each round's score / publish / combine
// tail (4.0 TB/s).  Here one workgroup takes one (kv group, sequence) and
// walks that sequence's own keys in 64-key chunks, the next chunk's K/V
// requested into a second register set before the current chunk's
// arithmetic; each wave keeps its own online softmax (m, l, O) over its 16
// keys of every chunk, so the loop has no barrier, no partial publish and no
// drain -- the four waves merge once through LDS at the end.  Only keys below
// the sequence's position are loaded (a short sequence in a batch streams
// only its own context).  Numerics: fp16 Q.K products summed in fp32 on MFMA,
// fp32 softmax and P.V as decode_attn_body; the merge order differs from the
// split kernels (a few fp32 ulps).
struct KvChunk {
    half8 kk[4];   // K, v_mfma_f32_16x16x32_f16 B layout: key 16 wid + c16, dims 32 s4 + 8 q4
    half8 vv[4];   // V rows 16 wid + 4 i + sub, dims dl .. dl + 8
};

__device__ __forceinline__ void kvc_issue(const uint16_t *kc, const uint16_t *vc, int c0, int kcap, bool want_v, KvChunk &r,
                                          bool nt) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int sub = lane >> 4, dl = (lane & 15) * 8, q4 = lane >> 4, c16 = lane & 15;
    const int kk = min(c0 + 16 * wid + c16, kcap);
#pragma unroll
    for (int s4 = 0; s4 < 4; s4++) r.kk[s4] = kv_load(kc + (long)kk * 128 + 32 * s4 + 8 * q4, nt);
    if (want_v)
#pragma unroll
        for (int i = 0; i < 4; i++) r.vv[i] = kv_load(vc + (long)min(c0 + 16 * wid + 4 * i + sub, kcap) * 128 + dl, nt);
}

struct SeqSt {
    float m0, m1, l0, l1;   // running max / sum per head (uniform in the wave)
    float o0[8], o1[8];     // this lane's partial O (its keys 4 i + sub, dims dl .. dl + 8)
};

// one 64-key chunk for this wave (keys c0 + 16 wid .. + 15)
__device__ __forceinline__ void kvc_step(const DecodeAttnArgs &a, const half8 *qa, const uint16_t *knew, const uint16_t *vnew,
                                         int c0, int pos, const KvChunk &r, SeqSt &st, float *sdst) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int q4 = lane >> 4, c16 = lane & 15, sub = lane >> 4, dl = (lane & 15) * 8;
    const int key = c0 + 16 * wid + c16;
    half8 kt[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; s4++) kt[s4] = key == pos ? *(const half8 *)&knew[32 * s4 + 8 * q4] : r.kk[s4];
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 4; s4++) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(qa[s4], kt[s4], acc, 0, 0, 0);
    // lanes 0-15 (q4 = 0): S[head r][key c16] in acc[r]
    const bool ok = q4 == 0 && key <= pos;
    const float s0 = ok ? acc[0] * a.scale : -INFINITY, s1 = ok ? acc[1] * a.scale : -INFINITY;
    if (sdst) {   // scores mode (front half of the exact attention, fa_exact.hip)
        if (ok) {
            sdst[key] = s0;
            sdst[(long)a.max_ctx + key] = s1;
        }
        return;
    }
    const float c0m = wave_max(s0), c1m = wave_max(s1);
    const float M0 = fmaxf(st.m0, c0m), M1 = fmaxf(st.m1, c1m);
    const float r0 = M0 == -INFINITY ? 1.f : expf(st.m0 - M0), r1 = M1 == -INFINITY ? 1.f : expf(st.m1 - M1);
    const float p0 = ok ? expf(s0 - M0) : 0.f, p1 = ok ? expf(s1 - M1) : 0.f;
    st.l0 = st.l0 * r0 + wave_sum(p0);
    st.l1 = st.l1 * r1 + wave_sum(p1);
    st.m0 = M0;
    st.m1 = M1;
#pragma unroll
    for (int e = 0; e < 8; e++) { st.o0[e] *= r0; st.o1[e] *= r1; }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int kl = 4 * i + sub;   // this lane's key of row i (lane kl of the score row holds its p)
        const float q0 = __shfl(p0, kl, 64), q1 = __shfl(p1, kl, 64);
        const half8 vr = c0 + 16 * wid + kl == pos ? *(const half8 *)&vnew[dl] : r.vv[i];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const float v = (float)vr[e];
            st.o0[e] = fmaf(v, q0, st.o0[e]);
            st.o1[e] = fmaf(v, q1, st.o1[e]);
        }
    }
}

// grid (n_kv_head, B): kv group g of sequence b, both of its query heads.
// FX = 1: ggml's fp16-accumulating attention in one launch -- the scores
// pass below writes both heads' scaled scores into LDS (dynamic, [2][max_ctx])
// instead of global memory, and after one barrier the four waves run
// fx_decode.h's chain (wave w: head 2 g + w / 2, dimensions 64 (w & 1) ..),
// exactly the arithmetic of decode_attn_seq_kernel<0> in scores mode followed
// by decode_attn_exact_pair_kernel, so the outputs are bit-identical; the
// kernel boundary, the scores' round trip through HBM and the second
// launch's ramp go, and one CU's workgroups overlap their K and V^T streams.
template <int FX>
__global__ __launch_bounds__(256, FX ? 4 : 1) void decode_attn_seq_kernel(DecodeAttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) float fxs[];
    __shared__ __attribute__((aligned(16))) uint16_t qs[2][128];
    __shared__ __attribute__((aligned(16))) uint16_t knew[128];
    __shared__ __attribute__((aligned(16))) uint16_t vnew[128];
    __shared__ float wst[4][2][2];                                  // per wave: (m, l) per head
    __shared__ __attribute__((aligned(16))) float wo[4][2][128];   // per wave: O per head
    stamp_start(a.stamp);
    const int g = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int QD = a.n_head * 128, KD = a.n_kv_head * 128;
    const int q4 = lane >> 4, c16 = lane & 15, sub = lane >> 4, dl = (lane & 15) * 8;
    // dev trace (QASR_DEV_TRACE, decode batches): row g + n_kv_head b: [start, q/k/v ready, scores done, chain done]
    auto mark = [&](int slot) {
        if (a.trace && tid == 0) a.trace[((long)b * a.n_kv_head + g) * 8 + slot] = rt_now();
    };
    mark(0);
    const long cbase = ((long)b * a.n_kv_head + g) * a.max_ctx;
    uint16_t *kc = a.kc + cbase * 128, *vc = a.vc + cbase * 128;
    const int pos = a.pos[b], nkv = pos + 1, kcap = min(pos, a.max_ctx - 1);
    const bool want_v = !FX && !a.scores;
    KvChunk A, B;
    kvc_issue(kc, vc, 0, kcap, want_v, A, a.kv_nt);
    // ---- the token's q / k / v: rms norm * weight + NEOX RoPE (decode_attn_body), new K/V row to the caches
    {
        const float *raw = a.qkv + (long)b * (QD + 2 * KD);
        const float *src = wid < 2 ? raw + (2 * g + wid) * 128 : raw + QD + (wid - 2) * KD + g * 128;
        const float x0 = src[lane], x1 = src[lane + 64];
        const float *nw = wid < 2 ? a.q_norm : a.k_norm;
        const float2 cs = *(const float2 *)(a.rope + ((long)pos * 64 + lane) * 2);
        if (wid < 3) {
            const double ss = wave_sum_d((double)(x0 * x0) + (double)(x1 * x1));
            const float scale = 1.0f / sqrtf((float)(ss / 128.0) + a.eps);
            const float y0 = fmul_rn(fmul_rn(x0, scale), nw[lane]), y1 = fmul_rn(fmul_rn(x1, scale), nw[lane + 64]);
            const uint16_t r0 = f_to_u16(y0 * cs.x - y1 * cs.y), r1 = f_to_u16(y0 * cs.y + y1 * cs.x);
            if (wid < 2) {
                qs[wid][lane] = r0;
                qs[wid][lane + 64] = r1;
            } else {
                knew[lane] = r0; knew[lane + 64] = r1;
                kc[(long)pos * 128 + lane] = r0;
                kc[(long)pos * 128 + lane + 64] = r1;
            }
        } else {
            const uint16_t v0 = f_to_u16(x0), v1 = f_to_u16(x1);
            vnew[lane] = v0; vnew[lane + 64] = v1;
            vc[(long)pos * 128 + lane] = v0;
            vc[(long)pos * 128 + lane + 64] = v1;
            uint16_t *t = a.vt + ((long)b * a.n_kv_head + g) * 128 * vt_ctx(a.max_ctx);
            t[vt_index(pos, lane)] = v0;
            t[vt_index(pos, lane + 64)] = v1;
        }
    }
    __syncthreads();
    mark(1);
    half8 qa[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; s4++)
        qa[s4] = c16 < 2 ? *(const half8 *)&qs[c16][32 * s4 + 8 * q4] : half8{0, 0, 0, 0, 0, 0, 0, 0};
    float *sdst = FX ? fxs : a.scores ? a.scores + ((long)b * a.n_head + 2 * g) * a.max_ctx : nullptr;
    SeqSt st;
    st.m0 = st.m1 = -INFINITY;
    st.l0 = st.l1 = 0.f;
#pragma unroll
    for (int e = 0; e < 8; e++) { st.o0[e] = 0.f; st.o1[e] = 0.f; }
    for (int c0 = 0; c0 < nkv; c0 += 128) {   // two chunks a trip, each prefetching the other set
        if (c0 + 64 < nkv) kvc_issue(kc, vc, c0 + 64, kcap, want_v, B, a.kv_nt);
        kvc_step(a, qa, knew, vnew, c0, pos, A, st, sdst);
        if (c0 + 64 >= nkv) break;
        if (c0 + 128 < nkv) kvc_issue(kc, vc, c0 + 128, kcap, want_v, A, a.kv_nt);
        kvc_step(a, qa, knew, vnew, c0 + 64, pos, B, st, sdst);
    }
    if constexpr (FX) {
        __syncthreads();   // both heads' scores in LDS; the new V^T row stored (this workgroup's own writes)
        mark(2);
        decode_attn_exact_body(a, 2 * g + (wid >> 1), b, wid & 1, fxs + (wid >> 1) * a.max_ctx);
        if (a.trace) __syncthreads();
        mark(3);
        stamp_end(a.stamp);
        return;
    }
    if (sdst) { stamp_end(a.stamp); return; }
    // ---- merge: lanes of equal dl hold partial O over their keys (sub = 0..3): sum over sub, then over waves
#pragma unroll
    for (int e = 0; e < 8; e++) {
        st.o0[e] += __shfl_xor(st.o0[e], 16, 64);
        st.o0[e] += __shfl_xor(st.o0[e], 32, 64);
        st.o1[e] += __shfl_xor(st.o1[e], 16, 64);
        st.o1[e] += __shfl_xor(st.o1[e], 32, 64);
    }
    if (sub == 0) {
        *(floatx4 *)&wo[wid][0][dl] = floatx4{st.o0[0], st.o0[1], st.o0[2], st.o0[3]};
        *(floatx4 *)&wo[wid][0][dl + 4] = floatx4{st.o0[4], st.o0[5], st.o0[6], st.o0[7]};
        *(floatx4 *)&wo[wid][1][dl] = floatx4{st.o1[0], st.o1[1], st.o1[2], st.o1[3]};
        *(floatx4 *)&wo[wid][1][dl + 4] = floatx4{st.o1[4], st.o1[5], st.o1[6], st.o1[7]};
    }
    if (lane == 0) {
        wst[wid][0][0] = st.m0; wst[wid][0][1] = st.l0;
        wst[wid][1][0] = st.m1; wst[wid][1][1] = st.l1;
    }
    __syncthreads();
    const int hh = tid >> 7, d = tid & 127;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; w++) M = fmaxf(M, wst[w][hh][0]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const float mw = wst[w][hh][0];
        const float f = mw == -INFINITY ? 0.f : expf(mw - M);
        L = fmaf(wst[w][hh][1], f, L);
        O = fmaf(wo[w][hh][d], f, O);
    }
    const float inv = L > 0.f ? 1.0f / L : 0.f;
    const float v = O * inv;
    const long e = (long)b * QD + (2 * g + hh) * 128 + d;
    if (a.outq) {   // quantised for the Q8_0 o-proj: a 32-block = 32 lanes of one wave
        float am = fabsf(v);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
        a.outq[e] = q8_quant(v, am);
        if ((d & 31) == 0) a.outd[e >> 5] = q8_scale(am);
    } else if (a.out32) a.out32[e] = v;
    else a.out[e] = f_to_u16(v);
    stamp_end(a.stamp);
}

int decode_stream_slots() {
    int nb = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(decode_attn_seq_kernel<0>), 256, 0) !=
            hipSuccess)
        return 0;
    return nb * cus;
}

// ------------------------------------------------- batch 1: QKV + attention
// One launch for the batch-1 QKV projection and the attention it feeds.
// Blocks [0, 512): the QKV GEMV (gemv1_kernel's arithmetic, K = 1024, 2 rows
// per wave, RMS norm / layer-0 embedding gather per wave), block q serving kv
// group q / 64 (its 256 q rows, 128 k rows, 128 v rows); outputs are stored
// write-through (sc1), every wave drains, and one lane counts the block into
// qcnt[group] (MI355X_MICROARCH.md hand-off table, row 1).  Blocks past 512:
// the group's attention splits, which issue their K/V loads before waiting
// for the count -- the K/V stream overlaps the projection instead of
// following a kernel boundary.  Dispatch order puts the QKV blocks first; the
// wait is bounded so no order can hang the GPU.
// Blocks past the attention splits (when att_done is set): the o-projection
// (gemv1 arithmetic, K = 2048, one row per wave, + residual): weights
// requested after a delay, a bounded wait for all kv groups' combiners
// (att_done replica block % 8), then the fp16 attention output and the
// residual row read with sc1 loads.  att_done is re-armed by the down-proj
// launch that follows (GemvArgs.zero8).
// One row a wave: 256 blocks of 4 rows.
constexpr int ORPW = 1, OPROJ_ROWS = 4 * ORPW;
__device__ __forceinline__ void oproj1_body(const GemvArgs o, const DecodeAttnArgs a, int j) {
    constexpr int K = 2048, NT = 4;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int row0 = j * OPROJ_ROWS + wid * ORPW;
    for (int i = 0; i < a.oproj_delay; i++) __builtin_amdgcn_s_sleep(8);
    half8 wv[ORPW][NT];
#pragma unroll
    for (int r = 0; r < ORPW; r++)
#pragma unroll
        for (int t = 0; t < NT; t++)
            wv[r][t] = __builtin_nontemporal_load((const half8 *)(o.W + (long)(row0 + r) * K + t * 512 + lane * 8));
    __shared__ int oready;
    if (threadIdx.x == 0) {
        int ok = 0;
        for (int it = 0; it < a.poll_limit; it++) {
            if (__hip_atomic_load(a.att_done + (j & 7) * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                (unsigned)a.n_kv_head) {
                ok = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(4);
        }
        if (a.fence) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (!ok) __hip_atomic_fetch_or(a.err, (unsigned)DEVERR_O_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        oready = ok;
    }
    __syncthreads();
    if (!oready) return;   // reported through the error word; x keeps its old rows
    u32x4 xv[NT];
    ld_sc1_x4_4(o.xh + lane * 8, xv);
    float res[ORPW];
#pragma unroll
    for (int r = 0; r < ORPW; r++)
        res[r] = __uint_as_float(__hip_atomic_load((const uint32_t *)(o.res + row0 + r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
    for (int r = 0; r < ORPW; r++) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const half8 h = __builtin_bit_cast(half8, xv[t]);
#pragma unroll
            for (int e = 0; e < 8; e++) acc = fmaf((float)wv[r][t][e], (float)h[e], acc);
        }
        acc = wave_sum(acc);
        if (lane == 0) o.out_f32[row0 + r] = fadd_rn(acc, res[r]);
    }
}

// Chain role of the fused exact attention (DecodeAttnArgs.fx): one workgroup
// per kv group g, wave w running query head 2g + w / 2, dimensions 64 (w % 2)
// + lane, with ggml's CPU flash-attention numerics (fx_chain.h; the same
// arithmetic as fa_exact.hip's decode_attn_exact_kernel, so the two launches
// are bit-identical).  V^T of keys below the position comes from the cache
// (earlier steps' rows; the first 128 keys requested at entry); the new key's
// v from its QKV granule.  The two heads' scores arrive as granules from the
// splits, gathered per DX_KC-key chunk into LDS (every thread polls its own
// 16-B granule pairs, bounded); each wave derives the chunk's weights from
// LDS into registers and runs the chain.  The output goes to the o-projection
// role as the split-K combiners' does (write-through, drained, att_done).
// eight 16-B sc1 loads at base + off[u] bytes (base uniform: the SGPR-pair
// address form, so the offsets cost one VGPR each), drained in the same asm
// block (no copy of an output can be scheduled before the data has landed)
__device__ __forceinline__ void ld_sc1_x4_8(const void *base, const uint32_t *off, u32x4 *v) {
    asm volatile(
        "global_load_dwordx4 %0, %8, %16 sc1\n\t"
        "global_load_dwordx4 %1, %9, %16 sc1\n\t"
        "global_load_dwordx4 %2, %10, %16 sc1\n\t"
        "global_load_dwordx4 %3, %11, %16 sc1\n\t"
        "global_load_dwordx4 %4, %12, %16 sc1\n\t"
        "global_load_dwordx4 %5, %13, %16 sc1\n\t"
        "global_load_dwordx4 %6, %14, %16 sc1\n\t"
        "global_load_dwordx4 %7, %15, %16 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
        : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), "v"(off[4]), "v"(off[5]), "v"(off[6]), "v"(off[7]), "s"(base)
        : "memory");
}
// chain workgroups of the fused launch: one a kv group (4 chain waves)
__host__ __device__ inline int fx_chain_wgs(int fx, int n_kv_head) { return fx ? n_kv_head : 0; }
// the chain role's LDS (fx1_chain_body: both heads): a layout of the fused
// launch's shared role buffer
struct alignas(16) ChainLds {
    float fsc[2][DX_KC / DX_B * FX_ST];
    uint16_t kmask[2][DX_KC / 16];
    float fwl[2];
};
// Phases (1) and (2) of a chain workgroup holding both query heads of kv group
// g (fx1_chain_body): the score granules of both heads -> LDS,
// then wave wid the weights of head wid / 2, half wid % 2 (C.fsc, C.kmask,
// C.fwl); returns that head's S.  n: keys (<= DX_KC); trow: its trace row.
__device__ __forceinline__ float fx1_gather_weights(const DecodeAttnArgs &a, const int g, const int n, ChainLds &C, const int trow) {
    auto &fsc = C.fsc;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int hh = wid >> 1, wu = __builtin_amdgcn_readfirstlane(wid & 1);
    auto mark = [&](int slot) {
        if (a.trace && tid == 0) a.trace[(long)trow * 8 + slot] = rt_now();
    };
    const uint32_t tag = gran_tag(a.pos[0], a.layer);
    const int np = (n + 1) >> 1;
    // (1) the score granules of both heads -> LDS: thread tid takes the 16-B
    //     pairs q = tid + 256 (u / 2) of head u % 2, all in flight together
    {
        const int ld = sgran_ld(a.max_ctx);
        const unsigned long long *gb = a.sgran + (long)(2 * g) * ld;   // uniform
        uint32_t go[DX_KC / 256];
#pragma unroll
        for (int u = 0; u < DX_KC / 256; u++) {
            const int q = tid + 256 * (u >> 1);
            go[u] = q < np ? (uint32_t)(((u & 1) * ld + 2 * q) * 8) : 0u;
        }
        u32x4 gv[DX_KC / 256];
        bool ok = false;
        int it = 0;
        unsigned long long tis = 0;   // (trace) the last poll's issue time
        for (; it < a.poll_limit; it++) {
            if (a.trace) tis = rt_now();
            ld_sc1_x4_8(gb, go, gv);
            ok = true;
#pragma unroll
            for (int u = 0; u < DX_KC / 256; u++) {
                const int q = tid + 256 * (u >> 1);
                if (q < np) ok = ok && gv[u][1] == tag && (2 * q + 1 >= n || gv[u][3] == tag);
            }
            if (__syncthreads_and(ok)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (a.trace && tid == 0) {   // rows 4010 + g: polls, the successful poll's issue time
            a.trace[(4010L + g) * 8 + 5] = (unsigned long long)it + 1;
            a.trace[(4010L + g) * 8 + 6] = tis;
        }
        if (!ok && tid == 0) __hip_atomic_fetch_or(a.err, (unsigned)DEVERR_SCORE_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int u = 0; u < DX_KC / 256; u++) {
            const int q = tid + 256 * (u >> 1), j = 2 * q;   // even: both keys in one 32-key row
            if (q < np)
                *(float2 *)&fsc[u & 1][(j >> 5) * FX_ST + (j & 31)] = make_float2(__uint_as_float(gv[u][0]), __uint_as_float(gv[u][2]));
        }
    }
    __syncthreads();
    mark(2);
    // (2) the weights of this wave's head, fx_weights_reg's arithmetic split
    //     over the head's two waves: both read the lane's 32 scores and take
    //     the maxima (a lane's batch holds a new maximum iff its maximum beats
    //     the exclusive prefix), wave wu computes the expf of keys 16 wu ..
    //     16 wu + 15 of every lane and writes them back over the scores.  The
    //     new key n - 1 gets weight 0 in LDS (a no-op for the chain loop, which
    //     reads the cache row another workgroup is writing) and its weight in
    //     fwl, applied once after the loop with vnew -- the same sequence of
    //     operations as fa_exact.hip's chain, so both launches agree bit for bit
    auto &fwl = C.fwl;
    auto &kmask = C.kmask;   // per head: new-maximum bit of every key
    float M, S;
    {
        float *row = fsc[hh] + lane * FX_ST;   // this lane's 32 keys
        float sv[DX_B];
#pragma unroll
        for (int i = 0; i < DX_B; i += 4) {
            const floatx4 r = *(const floatx4 *)&row[i];
#pragma unroll
            for (int e = 0; e < 4; e++) sv[i + e] = lane * DX_B + i + e < n ? r[e] : -INFINITY;
        }
        float lm = -INFINITY, lh = -INFINITY;
#pragma unroll
        for (int i = 0; i < DX_B / 2; i++) lh = fmaxf(lh, sv[i]);
#pragma unroll
        for (int i = DX_B / 2; i < DX_B; i++) lm = fmaxf(lm, sv[i]);
        lm = fmaxf(lm, lh);
        const float inc = wave_scan_max(lm);
        const float Mp0 = dpp_ninf<0x138, 0xF>(inc);   // exclusive prefix (lane 0: -inf; the chunk is the first)
        M = lane_f(inc, 63);
        float x[DX_B / 2];
        uint32_t kb = 0;
        // the wave's half of the lane's keys, indexed statically in each branch
        // (a select on wu became a wu-offset index into sv, which put sv in
        // scratch memory: a global-memory round trip before the chain)
        auto half = [&](auto hc) {
            constexpr int H = decltype(hc)::value;
            float Mq = H ? fmaxf(Mp0, lh) : Mp0;
#pragma unroll
            for (int i = 0; i < DX_B / 2; i++) {
                const float sc = sv[H * (DX_B / 2) + i];
                const bool gt = sc > Mq;
                const float e = expf(gt ? Mq - sc : sc - Mq);
                x[i] = gt ? -e : (sc != -INFINITY ? e : 0.0f);
                kb |= (uint32_t)gt << i;
                Mq = fmaxf(Mq, sc);
            }
        };
        if (wu) half(std::integral_constant<int, 1>{});
        else half(std::integral_constant<int, 0>{});
        kmask[hh][2 * lane + wu] = (uint16_t)kb;   // keys 32 lane + 16 wu ..: the slow path's 8-key groups
        __syncthreads();   // both waves have read their scores
        mark(6);
#pragma unroll
        for (int i = 0; i < DX_B / 2; i += 4) *(floatx4 *)&row[16 * wu + i] = floatx4{x[i], x[i + 1], x[i + 2], x[i + 3]};
        const int kl = n - 1;
        if (lane == (kl >> 5) && wu == ((kl >> 4) & 1)) {   // (its own store above: ordered)
            fwl[hh] = row[kl & 31];
            row[kl & 31] = 0.0f;
        }
        __syncthreads();
        mark(7);
        // the lane's sequential S = S * ms + vs over its 32 weights (key n - 1
        // read as 0 is S * 1 + 0 = S: its own term, the lane's last, goes after)
        const float wl = fwl[hh];
        float Sl = 0.0f;
#pragma unroll
        for (int i = 0; i < DX_B; i += 4) {
            const floatx4 r = *(const floatx4 *)&row[i];
#pragma unroll
            for (int e = 0; e < 4; e++) Sl = __builtin_signbit(r[e]) ? fadd_rn(fmul_rn(Sl, -r[e]), 1.0f) : fadd_rn(fmul_rn(Sl, 1.0f), r[e]);
        }
        if (lane == (kl >> 5)) Sl = __builtin_signbit(wl) ? fadd_rn(fmul_rn(Sl, -wl), 1.0f) : fadd_rn(fmul_rn(Sl, 1.0f), wl);
        const float Ml = fmaxf(Mp0, lm);
        S = wave_sum(Ml == -INFINITY ? 0.0f : Sl * expf(Ml - M));
    }
    return S;
}
__device__ __forceinline__ void fx1_chain_body(const DecodeAttnArgs &a, const int g, ChainLds &C) {
    auto &fsc = C.fsc;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int hh = wid >> 1, wu = __builtin_amdgcn_readfirstlane(wid & 1);
    const int d = 64 * wu + lane, loff = 8 * lane;
    const uint16_t *vt = a.vt + (long)g * 128 * vt_ctx(a.max_ctx) + 64 * wu * 8;   // batch 1: slot 0; the wave's key block 0
    // dev trace (QASR_DEV_TRACE): rows 4000 + g of the attention kernel's table:
    // [start, v ready, scores gathered, weights done, chain done, published,
    //  weights: expf pass done, weights stored]
    // (v ready comes after the weights: the new v is polled last)
    auto mark = [&](int slot) {
        if (a.trace && tid == 0) a.trace[(4000L + g) * 8 + slot] = rt_now();
    };
    mark(0);
    const int pos = a.pos[0], nkv = pos + 1;
    const uint32_t tag = gran_tag(pos, a.layer);
    const int QD = a.n_head * 128, KD = a.n_kv_head * 128;
    // V^T of the wave's 64 dimensions -> this CU's L2 while the scores are
    // computed: wave w pulls the key blocks kb = w / 2 (mod 2), so the four
    // waves cover their two dimension halves once; LDS-DMA pieces (no
    // register destination) into the wave's own 1 KiB of fsc, contents unused
    // (the first gather poll below drains them: its vmcnt(0) and barrier).
    // Without it the chain's V^T loads were HBM misses one 64-key buffer
    // ahead: ~40 cycles a key instead of ~12 (device trace, layer 14).
    if (a.fx_vpf & 2) {
        typedef __attribute__((address_space(3))) void lds_void_c;
        typedef __attribute__((address_space(1))) void glb_void_c;
        lds_void_c *dst = (lds_void_c *)((float *)fsc + wid * 256);
        for (int kb = hh; kb * 8 < nkv; kb += 2)
            __builtin_amdgcn_global_load_lds((glb_void_c *)(vt + (long)kb * 1024 + loff), dst, 16, 0, 0);
    }
    // one chunk: the launch is taken only while n_kv <= DX_KC (launch_qkv_attention1)
    const int n = nkv;
    const float S = fx1_gather_weights(a, g, n, C, 4000 + g);
    auto &fwl = C.fwl;
    auto &kmask = C.kmask;   // per head: new-maximum bit of every key
    mark(3);
    // the new key's v (this lane's dimension): its QKV granule, cast to fp16 as
    // the cache write is (long published by now: polled after the weights)
    uint16_t vnew = 0;
    {
        const unsigned long long *gp = a.gran + QD + KD + g * 128 + d;
        unsigned long long v = 0;
        bool ok = false;
        for (int it = 0; it < a.poll_limit; it++) {
            v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(v >> 32) == tag;
            if (__all(ok)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!__all(ok) && lane == 0) __hip_atomic_fetch_or(a.err, (unsigned)DEVERR_QKV_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vnew = f_to_u16(__uint_as_float((uint32_t)v));
    }
    mark(1);
    // (trace) shader clock against the 100 MHz counter over the chain: row 4010 + g
    const unsigned long long ck0 = a.trace ? clock64() : 0ull;
    f16 acc = 0;
    {
        // keys 0 .. n - 2 from V^T in 64-key steps (the last may run into key
        // n - 1 and past n: zero weights in fsc), then the new key
        const int nl = n - 1;
        u32x4 va[DX_Q / 8], vb[DX_Q / 8];
        floatx4 wa, wb;
        const int lastb = nl > 0 ? (nl - 1) >> 3 : 0;
        fx_loadQ(va, vt, loff, 0, lastb);
        fx_w8(fsc[hh], 0, wa, wb);
        for (int j0 = 0; j0 < nl; j0 += 2 * DX_Q) {
            fx_loadQ(vb, vt, loff, j0 + DX_Q, lastb);
            fx_step1_lds_m(va, j0, fsc[hh], fx_mask64(kmask[hh], j0), acc, wa, wb);
            if (j0 + DX_Q >= nl) break;
            fx_loadQ(va, vt, loff, j0 + 2 * DX_Q, lastb);
            fx_step1_lds_m(vb, j0 + DX_Q, fsc[hh], fx_mask64(kmask[hh], j0 + DX_Q), acc, wa, wb);
        }
        acc = fx_key_slow(acc, vnew, fwl[hh]);
    }
    mark(4);
    if (a.trace && lane == 0) {   // every wave: its chain's end (100 MHz) and shader cycles, rows 4020 + g, 4030 + g
        a.trace[(4020L + g) * 8 + wid] = rt_now();
        a.trace[(4030L + g) * 8 + wid] = clock64() - ck0;
    }
    if (a.trace && tid == 0) {
        a.trace[(4010L + g) * 8 + 0] = ck0;
        a.trace[(4010L + g) * 8 + 1] = clock64();
        a.trace[(4010L + g) * 8 + 2] = (unsigned long long)n;
    }
    // ggml: VKQ32 = fp32(VKQ16) * (1 / S); fp16 for the o-projection
    const float ov = (float)acc * (S == 0.0f ? 0.0f : 1.0f / S);
    const uint32_t h16 = f_to_u16(ov);
    const uint32_t hn = __shfl_xor(h16, 1, 64);
    uint16_t *out = a.out + (2 * g + hh) * 128 + d;
    if (a.att_done) {   // the o-proj blocks of this launch read it: write-through pairs, drained, one arrival per replica
        if ((lane & 1) == 0) __hip_atomic_store((uint32_t *)out, h16 | (hn << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (a.fence && tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (a.fence) __syncthreads();
        if (tid < 8) __hip_atomic_fetch_add(a.att_done + tid * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *out = (uint16_t)h16;
    }
    mark(5);
    if (a.trace && tid == 0) {   // (after the hand-off: one thread's 128 LDS reads took ~5 us before it)
        unsigned nk = 0, ng = 0;   // head 2g's new-maximum keys and slow 8-key groups
        for (int i = 0; i < DX_KC / 16; i++) {
            const unsigned m = kmask[0][i];
            nk += __builtin_popcount(m);
            ng += ((m & 0xffu) != 0) + ((m >> 8) != 0);
        }
        a.trace[(4010L + g) * 8 + 3] = nk;
        a.trace[(4010L + g) * 8 + 4] = ng;
    }
}

template <int SPL>
__global__ __launch_bounds__(256) void qkv_attn1_kernel(GemvArgs q, DecodeAttnArgs a, GemvArgs o) {
    constexpr int K = 1024, NT = 2, RPW = 2;
    // one LDS buffer for the roles that need one (a workgroup takes one role):
    // the split and chain layouts overlap instead of adding up
    constexpr size_t RLB = sizeof(SplitLds<SPL>) > sizeof(ChainLds) ? sizeof(SplitLds<SPL>) : sizeof(ChainLds);
    __shared__ __attribute__((aligned(16))) unsigned char role_lds[RLB];
    stamp_start(a.stamp);
    if (blockIdx.x >= 512) {
        // splits (kv group j % n_kv_head: blocks b and b + 8 share an XCD under
        // round-robin placement, so a group's splits and its chain workgroup
        // share one L2 -- speed only), the chain workgroups (exact attention),
        // the o-projection
        const int j = blockIdx.x - 512, nsp = a.grid_splits, nat = nsp * a.n_kv_head;   // grid_splits: this launch's splits
        const int nfx = fx_chain_wgs(a.fx, a.n_kv_head);
        if (j >= nat + nfx) oproj1_body(o, a, j - nat - nfx);
        else if (j >= nat) fx1_chain_body(a, j - nat, *reinterpret_cast<ChainLds *>(role_lds));
        else decode_attn_body<SPL, true>(a, j / a.n_kv_head, j % a.n_kv_head, 0, nsp, *reinterpret_cast<SplitLds<SPL> *>(role_lds));
        stamp_end(a.stamp);
        return;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int grp = blockIdx.x >> 6, loc = blockIdx.x & 63;
    if (q.trace && threadIdx.x == 0) q.trace[blockIdx.x * 8] = rt_now();
    const int QD = a.n_head * 128, KD = a.n_kv_head * 128;
    // the block's 8 rows: q rows of heads 2g, 2g+1, then k, then v of group g
    const int rbase = loc < 32 ? grp * 256 + loc * 8 : loc < 48 ? QD + grp * 128 + (loc - 32) * 8 : QD + KD + grp * 128 + (loc - 48) * 8;
    const int row0 = rbase + wid * RPW;
    const uint32_t gtag = a.gran ? gran_tag(a.pos[0], a.layer) : 0u;
    half8 wv[RPW][NT];
#pragma unroll
    for (int r = 0; r < RPW; r++)
#pragma unroll
        for (int t = 0; t < NT; t++)
            wv[r][t] = __builtin_nontemporal_load((const half8 *)(q.W + (long)(row0 + r) * K + t * 512 + lane * 8));
    float xf[NT][8];
    if (q.embd_ids) {   // layer 0: x = token_embd[id]
        const uint16_t *er = q.embd + (long)q.embd_ids[0] * K;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const half8 h = *(const half8 *)(er + t * 512 + lane * 8);
#pragma unroll
            for (int e = 0; e < 8; e++) xf[t][e] = (float)h[e];
        }
        if (q.x_store && blockIdx.x == 0 && wid == 0)   // write-through: the fused o-proj adds it as its residual
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int e = 0; e < 8; e++)
                    __hip_atomic_store((uint32_t *)(q.x_store + t * 512 + lane * 8 + e), __float_as_uint(xf[t][e]), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    } else {
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const float4 u = *(const float4 *)(q.x + t * 512 + lane * 8);
            const float4 v = *(const float4 *)(q.x + t * 512 + lane * 8 + 4);
            xf[t][0] = u.x; xf[t][1] = u.y; xf[t][2] = u.z; xf[t][3] = u.w;
            xf[t][4] = v.x; xf[t][5] = v.y; xf[t][6] = v.z; xf[t][7] = v.w;
        }
    }
    double ss = 0.0;   // ggml_rms_norm: double sum of fp32 squares
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int e = 0; e < 8; e++) ss += (double)(xf[t][e] * xf[t][e]);
    ss = wave_sum_d(ss);
    const float scale = 1.0f / sqrtf((float)(ss / K) + q.eps);
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const float4 u = *(const float4 *)(q.norm_w + t * 512 + lane * 8);
        const float4 v = *(const float4 *)(q.norm_w + t * 512 + lane * 8 + 4);
        const float w[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; e++) xf[t][e] = (float)f2h(fmul_rn(fmul_rn(xf[t][e], scale), w[e]));
    }
#pragma unroll
    for (int r = 0; r < RPW; r++) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int e = 0; e < 8; e++) acc = fmaf((float)wv[r][t][e], xf[t][e], acc);
        acc = wave_sum(acc);
        if (a.gran) {   // one 8-byte write-through {value, tag} store per output: the flag travels with the data
            if (lane == 0)
                __hip_atomic_store(a.gran + row0 + r, ((unsigned long long)gtag << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else if (lane == 0) {
            __hip_atomic_store((uint32_t *)(q.out_f32 + row0 + r), __float_as_uint(acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (a.gran) {   // nothing to drain or count
        if (q.trace && threadIdx.x == 0) q.trace[blockIdx.x * 8 + 1] = rt_now();
        stamp_end(a.stamp);
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (a.fence && threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (a.fence) __syncthreads();
    if (threadIdx.x < 8)   // one lane per replica of the group's counter
        __hip_atomic_fetch_add(a.qcnt + (grp * 8 + threadIdx.x) * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (q.trace && threadIdx.x == 0) q.trace[blockIdx.x * 8 + 1] = rt_now();
    stamp_end(a.stamp);
}

// batch <= 8 key split: cfg 64 / 128, else 64 up to 1.9k keys and 128 beyond (half the
// partials to combine, still >= 64 workgroups per 8 kv heads)
// (64-key splits up to 1.9k keys: with the fp16-V chain the split work is off the
// critical path and more, shorter splits publish their scores sooner -- configs[1]
// 256.2 -> 260.6 RTFx at ffn_wdelay 18, tools/r4/sweep.sh; past 1.9k keys the grid
// would outgrow the co-resident slots)
static int split1(int spl1, int grid_splits) { return spl1 == 64 || spl1 == 128 ? spl1 : grid_splits >= 30 ? 128 : 64; }

int launch_qkv_attention1(const GemvArgs &q, const DecodeAttnArgs &a, const GemvArgs *o, const FuseCfg &cfg, hipStream_t s, bool dry) {
    if (!cfg.qkv || !cfg.err || a.B != 1 || !a.qcnt || q.M != 1 || q.K != 1024 || q.Wd || !q.norm_w || q.xh || q.bias || q.res ||
        a.out32 || a.outq || q.N != a.n_head * 128 + 2 * a.n_kv_head * 128 || a.n_head != 2 * a.n_kv_head || a.n_kv_head * 64 != 512)
        return 0;
    const int spl1 = split1(cfg.spl1, a.grid_splits);   // as launch_decode_attention
    const int ns = (a.grid_splits * DSPLIT + spl1 - 1) / spl1;
    // the o-projection joins when it is the plain batch-1 f16 one (K = 2048, + residual)
    const bool with_o = cfg.o && o && a.att_done && o->M == 1 && o->K == 2048 && o->N == 1024 && o->xh && o->res &&
                        !o->Wd && !o->bias && !o->norm_w && o->xh == a.out;
    // every block of the launch must be co-resident (blocks wait on earlier
    // ones): fall back to separate launches for contexts that would not fit
    // (exact attention: n_kv_head chain workgroups too; they read the new v
    // from its granule, so the fused exact path needs the granule hand-off)
    // (fx_chain.h: one chain chunk)
    if (a.fx && (!a.gran || !a.sgran || ns * spl1 > DX_KC)) return 0;
    const int nfx = fx_chain_wgs(a.fx, a.n_kv_head);
    const int slots = spl1 == 128 ? cfg.slots_qkv128 : cfg.slots_qkv64;
    const int o_blocks = 1024 / OPROJ_ROWS;
    const bool fit_o = 512 + ns * a.n_kv_head + nfx + o_blocks <= slots;
    if (512 + ns * a.n_kv_head + nfx > slots) return 0;
    const bool with_o2 = with_o && fit_o;
    if (dry) return with_o2 ? 2 : 1;
    const dim3 grid(512 + ns * a.n_kv_head + nfx + (with_o2 ? o_blocks : 0));
    // K/V delay ~2 us: measured optimum on MI355X (round-1 delay sweep: 0 -> 236.3, 10 -> 232.0, 18 -> 240.3 ms decode)
    DecodeAttnArgs ad = a;
    ad.fuse_delay = cfg.qkv_delay;
    ad.oproj_delay = cfg.o_delay;
    ad.poll_limit = cfg.poll_limit;
    ad.fence = cfg.fence;
    ad.err = cfg.err;
    ad.grid_splits = ns;   // the kernel's split count
    ad.fx_vpf = cfg.fx_vpf;
    if (!with_o2) ad.att_done = nullptr;
    const GemvArgs qa = q;
    const GemvArgs oa = with_o2 ? *o : GemvArgs{};
    if (spl1 == 128) hipLaunchKernelGGL(qkv_attn1_kernel<128>, grid, dim3(256), 0, s, qa, ad, oa);
    else hipLaunchKernelGGL(qkv_attn1_kernel<DSPLIT>, grid, dim3(256), 0, s, qa, ad, oa);
    return with_o2 ? 2 : 1;
}

void launch_decode_attention(const DecodeAttnArgs &a, hipStream_t s) {
    if (a.B <= 0) return;
    if (a.B <= 8) {
        if (split1(a.spl1, a.grid_splits) == 128) {
            const int g2 = (a.grid_splits * DSPLIT + 127) / 128;
            hipLaunchKernelGGL(decode_attn_kernel<128>, dim3(g2, a.n_kv_head, a.B), dim3(256), 0, s, a);
        } else {
            hipLaunchKernelGGL(decode_attn_kernel<DSPLIT>, dim3(a.grid_splits, a.n_kv_head, a.B), dim3(256), 0, s, a);
        }
    } else if (a.stream_blocks > 0 && a.n_head == 2 * a.n_kv_head && a.n_kv_head * a.B >= a.stream_blocks / 2) {
        // batches that give every CU a sequence or more: one workgroup per (kv group, sequence)
        hipLaunchKernelGGL(decode_attn_seq_kernel<0>, dim3(a.n_kv_head, a.B), dim3(256), 0, s, a);
    } else {   // batches: longer splits (fewer workgroups and partials per sequence)
        if (a.spl_batch == 128) {
            const int g2 = (a.grid_splits * DSPLIT + 127) / 128;
            hipLaunchKernelGGL(decode_attn_kernel<128>, dim3(g2, a.n_kv_head, a.B), dim3(256), 0, s, a);
        } else {
            const int g4 = (a.grid_splits * DSPLIT + 255) / 256;
            hipLaunchKernelGGL(decode_attn_kernel<256>, dim3(g4, a.n_kv_head, a.B), dim3(256), 0, s, a);
        }
    }
}

// the one-launch exact attention of a decode batch where the per-sequence
// kernel is taken (launch_decode_attention) and both heads' scores fit the
// LDS budget; false = not covered (the caller runs scores + chain launches)
bool launch_decode_attention_exact_seq(const DecodeAttnArgs &a, hipStream_t s) {
    const size_t lds = (size_t)2 * a.max_ctx * sizeof(float);
    if (!a.fx_seq || a.B <= 8 || a.stream_blocks <= 0 || a.n_head != 2 * a.n_kv_head || a.n_kv_head * a.B < a.stream_blocks / 2 ||
        lds > 32768)
        return false;
    hipLaunchKernelGGL(decode_attn_seq_kernel<1>, dim3(a.n_kv_head, a.B), dim3(256), lds, s, a);
    return true;
}

int fused_slots_ffn();   // gemv.hip

void fused_slots(FuseCfg &cfg) {
    auto slots_of = [](const void *kernel) {
        int nb = 0, dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0) != hipSuccess)
            return 0;   // unknown capacity: never fuse
        return nb * cus;
    };
    cfg.slots_qkv64 = slots_of(reinterpret_cast<const void *>(qkv_attn1_kernel<DSPLIT>));
    cfg.slots_qkv128 = slots_of(reinterpret_cast<const void *>(qkv_attn1_kernel<128>));
    cfg.slots_ffn = fused_slots_ffn();
    cfg.slots_stream = decode_stream_slots();
}

int decode_split_len() { return DSPLIT; }
int decode_max_splits() { return 256; }

}  // namespace qasr
