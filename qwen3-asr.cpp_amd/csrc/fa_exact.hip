// fa_exact.hip -- decoder attention with ggml's CPU flash-attention numerics.
//
// ggml_flash_attn_ext on the CPU backend (the reference's Linux path,
// src/text_decoder.cpp:534-540; SURVEY.md §8(a) viii) walks the keys of one
// query row in order: s = (fp16 q . fp16 k) * scale; a new maximum rescales
// the fp16 V accumulator (ggml_vec_scale_f16: y = fp16(y * ms)), every key
// adds v * vs into it (ggml_vec_mad_f16: y = fp16(fma(v, vs, y))), and
// S = S * ms + vs in fp32; the output is fp32(acc) * (1 / S).  The fp16
// rounding after every key makes the result order-dependent: it cannot be
// split over keys, so each (query, head, dimension) is one sequential chain.
// At a 1.2k-token prompt that rounding moves the attention output by ~1 % of
// its scale against an fp32 accumulator (tests/test_gpu_full.py, configs[1]).
//
// Reproduced exactly: the chain -- the running maximum and each key's
// (ms, vs) (a prefix maximum is exact, so a wave scan gives the sequential
// loop's values) and every fp16 rounding of the accumulator, in key order.
// Not reproduced: the scores' fp32 summation order (MFMA vs
// ggml_vec_dot_f16) and S, summed here in parallel as sum_k exp(s_k - M) (the
// sequential S * ms + vs up to fp32 rounding, ~1e-7 relative) -- both far
// below the fp16 accumulator's own rounding.
//
// The chain step is v_fma_mix_f32 (fp16 v and accumulator, fp32 vs, one fp32
// rounding) and then an fp16 conversion.  LLVM folds fptrunc(fma) into
// v_fma_mixlo_f16, which rounds once, straight to fp16 (dev_common.h rn32).
// A pair of values converted as a vector becomes v_cvt_pk_f16_f32 and does not
// fold (this file is built with -fno-slp-vectorize, so the two fmas stay mix
// instructions on the fp16 halves instead of one v_pk_fma_f32 behind four
// conversions); the single-value form converts in inline asm.
//
// Prefill: one workgroup = 16 query rows of one head (one MFMA column each);
// keys in chunks of PX_KC: (1) scores on MFMA -> LDS, (2) wave w derives the
// weights of its rows 2w, 2w + 1 (one half-wave a row) -> LDS, (3) wave w
// runs the chain of those rows with two dimensions per lane, V staged in LDS
// once for all rows.
// Decode: launch_decode_attention in scores mode writes the scaled scores;
// then one workgroup per (query head, sequence): both waves derive the
// weights, each runs the chain for 64 dimensions, one per lane (the shortest
// per-key latency: v_fma_mix_f32, one wait state, v_cvt_f16_f32), V from the
// V^T cache copy (kernels.h vt_ctx) in 16-B loads of 8 keys.
//
// Measured per-key costs (tools/micro/chain_lat.hip, one wave): fp32 fma
// chain 9.8 cycles, one dimension 13.3, two dimensions 14.0, four rows x two
// dimensions 62 -- a wave issues a VALU instruction every ~5 cycles, and
// more waves per SIMD do not slow each other.
#include "dev_common.h"
#include "fx_chain.h"
#include "fx_decode.h"
#include "kernels.h"

namespace qasr {

#define PX_ROWS 16   // prefill query rows per workgroup
#define PX_KC 128    // prefill keys per chunk
#ifndef FX_B
#define FX_B 16      // chain batch: keys whose V and weights are in registers together
#endif

// ggml_vec_mad_f16 on two dimensions packed in one dword: fp16(fma(v, vs, acc))
__device__ __forceinline__ half2v fx_mad2(half2v acc, uint32_t v, float vs) {
    const half2v vv = __builtin_bit_cast(half2v, v);
    const float f0 = fmaf((float)vv.x, vs, (float)acc.x);
    const float f1 = fmaf((float)vv.y, vs, (float)acc.y);
    return __builtin_convertvector((floatx2){f0, f1}, half2v);
}
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// ------------------------------------------------------------------ prefill
// grid (ceil(max_len / 16), n_head, n_seq), block 512: rows q0 .. q0 + 15,
// longest rows first; wave w owns rows 2w, 2w + 1 (two rows a wave: the chain
// is issue-bound at ~5 cycles an instruction per wave, so fewer rows per wave
// shorten the longest workgroups, which bound the launch).  Per chunk the V
// rows go global -> LDS by LDS-DMA (global_load_lds_dwordx4, issued first,
// landing while the scores and weights are computed): one copy serves all
// 16 rows.
#define PX_SCS (PX_KC + 4)   // score row stride (floats): the MFMA writes of 16 rows hit 16 banks
#define PX_W 8               // waves per workgroup
#define PX_R (PX_ROWS / PX_W)
#ifndef PX_MINW
#define PX_MINW 1   // minimum waves per SIMD asked of the register allocator
#endif
// Round 6: the same arithmetic per (row, key) as the round-5 kernel (kept as
// tools/micro/px_v0.h, the A/B baseline of tools/micro/px_bench) -- scores,
// (ms, vs), S and the chain -- in 24 % fewer VALU instructions (the kernel is
// VALU-issue bound: tools/micro/px_bench PMC, ~80 % of its cycles issue VALU):
//  * the weights of the wave's two rows at once, lanes 0-31 row 2w and 32-63
//    row 2w + 1, four keys a lane: one LDS read of the four scores, a 32-lane
//    prefix-maximum scan, one shared sum tree -- S is the same balanced
//    pairwise sum over the chunk's 128 keys in key order (lane pairs there,
//    lane quads here: the same tree), so the same fp32 value;
//  * expf(gt ? Mp - s : s - Mp) as expf(-|s - Mp|) (a - b = -(b - a) exactly)
//    through px_expf_nonpos, the device expf without its overflow clamp;
//  * one word a key: vs, or -ms at a new maximum (vs = 1 there); the
//    new-maximum keys of each 16-key batch as a bit mask per row, so the
//    chain scales the accumulator only at those keys (ggml's order: scale,
//    then the mad with vs = 1), by v_fma_mix_f32 with a -0 addend (= the fp32
//    product) -- the other keys of such a batch keep the 3-instruction body;
//  * the chunk's partial last batch runs the full body with v = -0 past the
//    wave's last key (fma(-0, vs, acc) = acc exactly, as skipping the key);
//  * wave-uniform loop bounds (the wave index through readfirstlane) and no
//    barrier between a wave's weights and its chain (its own rows only).
// Bit-identical to the round-5 kernel on every tools/micro/px_bench case
// (causal batches, a key-0 attention sink, cached prefixes, the aligner's
// fp32 scores); 1.13-1.31x faster (2.57 -> 1.99 ms a layer at 128 x 405).
//
// fp16(fp32(acc) * ms) with ms = -x (v_fma_mix_f32 negates its f32 operand)
__device__ __forceinline__ half2v fx_scale2n(half2v acc, float x) {
    float lo, hi;
    const float nz = -0.0f;
    asm("v_fma_mix_f32 %0, %1, -%2, %3 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(acc), "v"(x), "v"(nz));
    asm("v_fma_mix_f32 %0, %1, -%2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(hi) : "v"(acc), "v"(x), "v"(nz));
    return __builtin_convertvector((floatx2){lo, hi}, half2v);
}
// expf at x <= 0 (or NaN): the instruction sequence of this ROCm's device
// expf (__ocml_exp_f32: x log2(e) split in two fp32 parts, v_exp_f32 of the
// fraction, v_ldexp_f32 by the rounded integer part, 0 below -103.28) without
// its overflow clamp, which never applies at x <= 0; the same bits as expf on
// every x <= 0 (tools/micro/px_bench checks all 2^31 of them)
__device__ __forceinline__ float px_expf_nonpos(float x) {
    const float l2e = __uint_as_float(0x3fb8aa3bu), l2e_lo = __uint_as_float(0x32a5705fu);
    const float ph = x * l2e;
    float pl = __builtin_fmaf(x, l2e, -ph);
    pl = __builtin_fmaf(x, l2e_lo, pl);
    const float e = __builtin_rintf(ph);
    const float f = (ph - e) + pl;
    const float r = __builtin_ldexpf(__builtin_amdgcn_exp2f(f), (int)e);
    return x < __uint_as_float(0xc2ce8ed0u) ? 0.0f : r;
}
// px_expf_nonpos against the device expf on every x <= 0: all 2^31 bit
// patterns with the sign set, and +0 (qasr_check_expf_nonpos, a GPU test)
__global__ __launch_bounds__(256) void expf_nonpos_check_kernel(unsigned long long *bad) {
    const uint32_t base = (blockIdx.x * 256u + threadIdx.x) * 16u;
    unsigned long long nb = 0;
    for (uint32_t k = 0; k < 16; k++) {
        const float x = __uint_as_float((base + k) | 0x80000000u);
        const float a = expf(x), b = px_expf_nonpos(x);
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) nb++;
    }
    if (base == 0 && __float_as_uint(expf(0.0f)) != __float_as_uint(px_expf_nonpos(0.0f))) nb++;
    if (nb) atomicAdd(bad, nb);
}
hipError_t check_expf_nonpos(unsigned long long *mismatches) {
    unsigned long long *d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(*d));
    if (e != hipSuccess) return e;
    if ((e = hipMemset(d, 0, sizeof(*d))) == hipSuccess) {
        hipLaunchKernelGGL(expf_nonpos_check_kernel, dim3(1u << 19), dim3(256), 0, 0, d);
        if ((e = hipGetLastError()) == hipSuccess) e = hipMemcpy(mismatches, d, sizeof(*d), hipMemcpyDeviceToHost);
    }
    (void)hipFree(d);
    return e;
}
// the chain step of one row at key i of a batch whose new-maximum keys are
// the bits of mk: x = the key's word (vs, or -ms at a new maximum)
__device__ __forceinline__ half2v fx_key(half2v acc, uint32_t v, float x, uint32_t mk, int i) {
    float vs = x;
    if ((mk >> i) & 1u) {   // uniform
        acc = fx_scale2n(acc, x);
        vs = 1.0f;
    }
    return fx_mad2(acc, v, vs);
}

template <bool F32S>   // fp32 Q / K scores (the aligner)
__global__ __launch_bounds__(64 * PX_W, PX_MINW) void prefill_attn_exact_kernel(PrefillAttnArgs a) {
    __shared__ __attribute__((aligned(16))) float sc[PX_ROWS][PX_SCS];   // scores, then vs / -ms
    __shared__ __attribute__((aligned(16))) uint32_t fl[PX_KC / FX_B][PX_ROWS];   // new-maximum key masks
    __shared__ __attribute__((aligned(16))) uint32_t vsh[PX_KC * 64];
    static_assert(FX_B == 16 && PX_KC == 128 && PX_R == 2, "four keys a lane, four lanes a batch, two rows a wave");
    const int sq = blockIdx.z, h = blockIdx.y;
    const int L = a.seq_len[sq];
    const int nqb = (a.max_len + PX_ROWS - 1) / PX_ROWS;
    const int q0 = (nqb - 1 - (int)blockIdx.x) * PX_ROWS;
    if (q0 >= L) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, ql = lane & 15;
    const int hk = h / (a.n_head / a.n_kv_head);
    const int row0 = a.seq_row0[sq];
    const int QD = a.n_head * 128;
    const long cbase = ((long)a.seq_slot[sq] * a.n_kv_head + hk) * a.max_ctx;
    const uint16_t *kc = a.kc + cbase * 128, *vc = a.vc + cbase * 128;
    half8 qf[4];
    const bool qv = q0 + ql < L;
#pragma unroll
    for (int s = 0; s < 4; s++)
        qf[s] = qv ? *(const half8 *)(a.q + (long)(row0 + q0 + ql) * QD + h * 128 + 32 * s + 8 * g) : half8{};
    const int P0 = a.seq_pos0 ? a.seq_pos0[sq] : 0;
    const int lim = qv ? P0 + q0 + ql : -1;
    const int kend = min(P0 + L, P0 + q0 + PX_ROWS);
    const int r0 = PX_R * wid;
    const int wlast = min(P0 + L - 1, P0 + q0 + r0 + PX_R - 1);
    // weights lanes: half hf = row r0 + hf, keys 4 l32 .. 4 l32 + 3 of the chunk
    const int hf = lane >> 5, l32 = lane & 31, myrow = r0 + hf;
    float M = -INFINITY, S = 0.0f;   // row myrow's (uniform in each half)
    half2v acc[PX_R];
#pragma unroll
    for (int r = 0; r < PX_R; r++) acc[r] = half2v{0, 0};
    for (int c0 = 0; c0 < kend; c0 += PX_KC) {
        const int n = min(PX_KC, kend - c0);
        __syncthreads();   // the previous chunk's chains are done with sc / fl / vsh
#pragma unroll
        for (int it = wid; it < PX_KC / 4; it += PX_W)
            __builtin_amdgcn_global_load_lds((glb_void *)(vc + (long)(c0 + 4 * it + (lane >> 4)) * 128 + 8 * (lane & 15)),
                                             (lds_void *)(vsh + it * 256), 16, 0, 0);
        // (1) scores: 16-key tile t = wid (as prefill_attn_exact_kernel)
        if constexpr (F32S) {
            const int t = wid;
            if (t * 16 < n) {
                const int key = min(c0 + t * 16 + ql, kend - 1);
                const float *kr = a.k32 + (long)(row0 + key) * (a.n_kv_head * 128) + hk * 128 + 32 * g;
                const float *qr = a.q32 + (long)(row0 + min(q0 + ql, L - 1)) * QD + h * 128 + 32 * g;
                float kv[32], qv2[32];
#pragma unroll
                for (int i = 0; i < 32; i += 4) {
                    *(float4 *)&kv[i] = *(const float4 *)&kr[i];
                    *(float4 *)&qv2[i] = qv ? *(const float4 *)&qr[i] : float4{0.f, 0.f, 0.f, 0.f};
                }
                floatx4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < 32; kk += 2) {
                    s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[kk], qv2[kk], s0, 0, 0, 0);
                    s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[kk + 1], qv2[kk + 1], s1, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int k = c0 + t * 16 + 4 * g + i;
                    sc[ql][t * 16 + 4 * g + i] = k <= lim ? (s0[i] + s1[i]) * a.scale : -INFINITY;
                }
            }
        } else {
            const int t = wid;
            const int key = min(c0 + t * 16 + ql, kend - 1);
            half8 kf[4];
#pragma unroll
            for (int s = 0; s < 4; s++) kf[s] = *(const half8 *)(kc + (long)key * 128 + 32 * s + 8 * g);
            if (t * 16 < n) {
                floatx4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 4; s++) sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], qf[s], sacc, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int k = c0 + t * 16 + 4 * g + i;
                    sc[ql][t * 16 + 4 * g + i] = k <= lim ? sacc[i] * a.scale : -INFINITY;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's V pieces landed
        __syncthreads();   // every score and every V piece in LDS
        // (2) weights of rows r0, r0 + 1: fx_weights' arithmetic per key
        {
            const float4 s4 = *(const float4 *)&sc[myrow][4 * l32];
            float v[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (4 * l32 + i >= n) v[i] = -INFINITY;
            float inc = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
            // inclusive prefix maximum over each half's 32 lanes: row_shr 1, 2, 4, 8, then row 0's
            // (row 2's) last lane into row 1 (row 3)
            inc = fmaxf(inc, dpp_ninf<0x111, 0xF>(inc));
            inc = fmaxf(inc, dpp_ninf<0x112, 0xF>(inc));
            inc = fmaxf(inc, dpp_ninf<0x114, 0xF>(inc));
            inc = fmaxf(inc, dpp_ninf<0x118, 0xF>(inc));
            inc = fmaxf(inc, dpp_ninf<0x142, 0xA>(inc));
            float ex = dpp_ninf<0x138, 0xF>(inc);   // wave_shr:1: the exclusive prefix
            if (l32 == 0) ex = -INFINITY;           // (lane 32 got row 2w's total)
            float Mp = fmaxf(M, ex);
            const float tA = lane_f(inc, 31), tB = lane_f(inc, 63);
            const float Mn = fmaxf(M, hf ? tB : tA);
            float w4[4], t[4];
            uint32_t gtm = 0, need = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                // fx_weights' per-key values: a new maximum gives ms = expf(Mp - s) (0 before the
                // row's first key) and vs = 1, any other key vs = expf(s - Mp); a masked key (s = -inf)
                // of a valid row has a finite Mp (its key 0 is never masked), so expf gives its weight
                // 0 without a test -- rows past the sequence (every key masked) get NaN weights, and
                // their outputs are never stored
                const float s = v[i];
                const bool gt = s > Mp;
                const float e = px_expf_nonpos(-fabsf(s - Mp));
                w4[i] = gt ? -e : e;   // the key's word: -ms, or vs
                t[i] = gt ? 1.0f : e;
                Mp = fmaxf(Mp, s);
                gtm |= (gt ? 1u : 0u) << i;
                need |= (Mp != Mn ? 1u : 0u) << i;
            }
            *(float4 *)&sc[myrow][4 * l32] = make_float4(w4[0], w4[1], w4[2], w4[3]);
            if (need) {   // keys before a later new maximum of the chunk: their own S term
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if ((need >> i) & 1) t[i] = px_expf_nonpos(v[i] - Mn);
            }
            float ps = (t[0] + t[1]) + (t[2] + t[3]);
            ps = row16_sum(ps);
            const float psA = lane_f(ps, 0) + lane_f(ps, 16), psB = lane_f(ps, 32) + lane_f(ps, 48);
            ps = hf ? psB : psA;
            S = (M == -INFINITY ? 0.0f : M == Mn ? S : S * px_expf_nonpos(M - Mn)) + ps;
            M = Mn;
            // batch b = l32 / 4: its 16-bit new-maximum key mask from the four lanes' nibbles
            uint32_t nib = gtm << (4 * (l32 & 3));
            nib |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nib, 0xB1, 0xF, 0xF, true);
            nib |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nib, 0x4E, 0xF, 0xF, true);
            if ((l32 & 3) == 0) fl[l32 >> 2][myrow] = nib;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (LDS ops of one wave complete in order)
        __builtin_amdgcn_wave_barrier();
        // (3) the chain, up to the wave's longest row
        const int nw = min(n, wlast + 1 - c0);
        const uint32_t *vl = vsh + lane;
        for (int j0 = 0; j0 < nw; j0 += FX_B) {
            uint32_t v[FX_B];
#pragma unroll
            for (int i = 0; i < FX_B; i++) v[i] = vl[(j0 + i) * 64];
            const int nb = nw - j0;
            if (nb < FX_B) {
#pragma unroll
                for (int i = 0; i < FX_B; i++)
                    if (i >= nb) v[i] = 0x80008000u;   // -0: fma(-0, vs, acc) = acc
            }
            const uint32_t mA = __builtin_amdgcn_readfirstlane(fl[j0 / FX_B][r0]);
            const uint32_t mB = __builtin_amdgcn_readfirstlane(fl[j0 / FX_B][r0 + 1]);
            const float *x0 = sc[r0] + j0, *x1 = sc[r0 + 1] + j0;
            if ((mA | mB) == 0) {
#pragma unroll
                for (int i = 0; i < FX_B; i++) {
                    acc[0] = fx_mad2(acc[0], v[i], x0[i]);
                    acc[1] = fx_mad2(acc[1], v[i], x1[i]);
                }
            } else {
                // both rows' words in registers first (left to itself, the compiler sinks each load
                // into its key's branch: an LDS round trip a key)
                floatx4 xa[FX_B / 4], xb[FX_B / 4];
#pragma unroll
                for (int i = 0; i < FX_B / 4; i++) {
                    xa[i] = *(const floatx4 *)(x0 + 4 * i);
                    xb[i] = *(const floatx4 *)(x1 + 4 * i);
                }
#pragma unroll
                for (int i = 0; i < FX_B / 4; i++) asm volatile("" : "+v"(xa[i]), "+v"(xb[i]));
                // four-key groups: a group without a new maximum runs the plain body, the others test
                // each key (one new maximum a batch is the common case past a row's first keys)
#pragma unroll
                for (int gq = 0; gq < FX_B / 4; gq++) {
                    const uint32_t ga = (mA >> (4 * gq)) & 15u, gb = (mB >> (4 * gq)) & 15u;
                    if ((ga | gb) == 0) {
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            acc[0] = fx_mad2(acc[0], v[4 * gq + k], xa[gq][k]);
                            acc[1] = fx_mad2(acc[1], v[4 * gq + k], xb[gq][k]);
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            acc[0] = fx_key(acc[0], v[4 * gq + k], xa[gq][k], ga, k);
                            acc[1] = fx_key(acc[1], v[4 * gq + k], xb[gq][k], gb, k);
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < PX_R; r++) {
        const int q = q0 + r0 + r;
        if (q >= L) continue;
        // S of row r0 + r lives in half r
        const float Sr = lane_f(S, 32 * r);
        const float inv = Sr == 0.0f ? 0.0f : 1.0f / Sr;
        const float o0 = (float)acc[r].x * inv, o1 = (float)acc[r].y * inv;
        const long o = (long)(row0 + q) * QD + h * 128 + 2 * lane;
        if (a.out32) {
            a.out32[o] = o0;
            a.out32[o + 1] = o1;
        } else {
            *(uint32_t *)(a.out + o) = (uint32_t)f_to_u16(o0) | ((uint32_t)f_to_u16(o1) << 16);
        }
    }
}

void launch_prefill_attention_exact(const PrefillAttnArgs &a, hipStream_t s) {
    if (a.n_seq <= 0 || a.max_len <= 0) return;
    dim3 grid((a.max_len + PX_ROWS - 1) / PX_ROWS, a.n_head, a.n_seq);
    if (a.k32) hipLaunchKernelGGL(prefill_attn_exact_kernel<true>, grid, dim3(64 * PX_W), 0, s, a);
    else hipLaunchKernelGGL(prefill_attn_exact_kernel<false>, grid, dim3(64 * PX_W), 0, s, a);
}

// grid (n_head, B), block 128: one query head per workgroup
__global__ __launch_bounds__(128) void decode_attn_exact_kernel(DecodeAttnArgs a) {
    stamp_start(a.stamp);
    decode_attn_exact_body(a, blockIdx.x, blockIdx.y, threadIdx.x >> 6,
                           a.scores + ((long)blockIdx.y * a.n_head + blockIdx.x) * a.max_ctx);
    stamp_end(a.stamp);
}

// grid (n_head / 2, B), block 256: the two query heads 2x, 2x + 1 of one kv
// group (GQA 2:1) in one workgroup -- waves 0/1 and 2/3 stream the same V^T
// rows close together in time, so the second read is served by the CU's
// caches instead of HBM (one head per workgroup read every V row twice from
// memory: the Q8_0 batch-64 decode's largest kernel, memory-bound).  Same
// per-wave arithmetic, so the outputs are bit-identical.
__global__ __launch_bounds__(256) void decode_attn_exact_pair_kernel(DecodeAttnArgs a) {
    stamp_start(a.stamp);
    const int wid = threadIdx.x >> 6;
    const int h = 2 * blockIdx.x + (wid >> 1);
    decode_attn_exact_body(a, h, blockIdx.y, wid & 1, a.scores + ((long)blockIdx.y * a.n_head + h) * a.max_ctx);
    stamp_end(a.stamp);
}

void launch_decode_attention_exact(const DecodeAttnArgs &a, hipStream_t s) {
    if (a.B <= 0) return;
    // (measured on configs[2], Q8_0 64 x 30 s: decode 285.7 -> 267.2 ms, tools/experiments.sh fxpair)
    if (a.n_head % 2 == 0 && (a.n_head / a.n_kv_head) % 2 == 0)
        hipLaunchKernelGGL(decode_attn_exact_pair_kernel, dim3(a.n_head / 2, a.B), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(decode_attn_exact_kernel, dim3(a.n_head, a.B), dim3(128), 0, s, a);
}

}  // namespace qasr
