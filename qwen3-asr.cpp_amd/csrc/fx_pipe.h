// fx_pipe.h -- the decode-step chain of ggml's CPU flash attention with the
// weights derived on the fly, one 64-key buffer at a time (round 4).
//
// Same arithmetic as fx_chain.h (src/text_decoder.cpp:534-540 through
// ggml_flash_attn_ext's CPU loop): per key s = q.k * scale; a new running
// maximum rescales the fp16 accumulator (fp16(fp32(acc) * ms)); every key adds
// v * vs (fp16(fma(fp32(v), vs, fp32(acc))), rounded to fp32 and then to
// fp16).  What changes is where the weights come from:
//
//  * a wave derives the weights of 64 keys at a time, lane = key (one wave
//    scan for the running maximum, one expf a lane), one buffer ahead of the
//    chain -- so the chain starts as soon as the first 64 scores exist instead
//    of after a pass over the whole context, and the scores can arrive while
//    the chain runs (the batch-1 fused launch polls them per buffer);
//  * the chain reads key k's weight as an SGPR operand of v_fma_mix_f32: the
//    8 weights of the next 8-key group are moved into SGPRs by v_readlane
//    inside the current group's asm block, in the slots the mix -> convert
//    dependency leaves idle (no LDS round trip, no wait on a load);
//  * the new-maximum bits of a buffer are its ballot (uniform), so a group
//    holding a maximum takes the slow block without a mask read.
//
// S (the softmax denominator) is kept per lane -- lane l sums the keys
// 64 b + l, rescaled to the running maximum after every buffer -- and summed
// over the wave once at the end: not ggml's sequential fp32 S * ms + vs (that
// order is not reproduced anywhere in this engine; ~1e-7 relative).
#pragma once
#include "dev_common.h"
#include "fx_chain.h"

namespace qasr {

// the weights of one 64-key buffer from its scores (lane = key j0 + lane;
// -inf: masked or past the keys).  Signed as fx_chain.h: w = vs where the key
// is not a new maximum, w = -ms where it is (vs = 1 there); keys with -inf get
// weight 0.  M: running maximum (in/out); Sl: this lane's share of S, rescaled
// to the new maximum; returns the weight, m64 = the buffer's new-maximum bits.
// A buffer without a new maximum (all but a few: a running maximum over n
// scores has ~ln n records) takes one expf a lane and no scan; the full path
// gives the same values there (Mp = Mn = M, expf(0) = 1).
__device__ __forceinline__ float fxp_weights(float s, float &M, float &Sl, unsigned long long &m64) {
    m64 = __ballot(s > M);
    if (m64 == 0ull) {   // (uniform) s <= M on every lane
        const float w = s != -INFINITY ? expf(s - M) : 0.0f;
        Sl += w;
        return w;
    }
    const float inc = wave_scan_max(s);
    const float Mp = fmaxf(M, dpp_ninf<0x138, 0xF>(inc));   // exclusive prefix (lane 0: M)
    const float Mn = fmaxf(M, lane_f(inc, 63));
    const bool gt = s > Mp;
    const float e = expf(gt ? Mp - s : s - Mp);
    m64 = __ballot(gt);
    Sl = (M == -INFINITY ? 0.0f : Sl * expf(M - Mn)) + (s == -INFINITY ? 0.0f : expf(s - Mn));
    M = Mn;
    return gt ? -e : (s != -INFINITY ? e : 0.0f);
}

// DX_Q keys of V^T from key block j0 / 8 through a buffer descriptor (vt:
// the wave's key block 0; voff = 16 lane bytes): the block offset is an SGPR
// (soffset), so the loads cost no VALU address arithmetic; blocks past lastb
// re-read lastb (as fx_loadQ)
__device__ __forceinline__ void fxp_loadQ(u32x4 *v, __amdgpu_buffer_rsrc_t rs, int voff, int j0, int lastb) {
#pragma unroll
    for (int i = 0; i < DX_Q / 8; i++)
        v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, min(j0 / 8 + i, lastb) * 2048, 0));
}

// one 8-key group of the chain: v = 8 keys of this lane's dimension (fp16
// pairs), w0..w7 = their weights in SGPRs; reads lanes LN .. LN + 7 of wn (the
// next group's weights, lane = key) into n0..n7 on the way.
#define FXP_MIX(VI, W, SEL) "v_fma_mix_f32 %[t], " VI ", " W ", %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
#define FXP_RL(N, L) "v_readlane_b32 " N ", %[wn], " #L "\n\t"
#define FXP_CVT "v_cvt_f16_f32 %[a], %[t]\n\t"
#define FXP_FAST_BODY(L0, L1, L2, L3, L4, L5, L6, L7)                                                               \
    FXP_MIX("%[v0]", "%[w0]", "0") FXP_RL("%[n0]", L0) FXP_CVT FXP_MIX("%[v0]", "%[w1]", "1") FXP_RL("%[n1]", L1) FXP_CVT \
    FXP_MIX("%[v1]", "%[w2]", "0") FXP_RL("%[n2]", L2) FXP_CVT FXP_MIX("%[v1]", "%[w3]", "1") FXP_RL("%[n3]", L3) FXP_CVT \
    FXP_MIX("%[v2]", "%[w4]", "0") FXP_RL("%[n4]", L4) FXP_CVT FXP_MIX("%[v2]", "%[w5]", "1") FXP_RL("%[n5]", L5) FXP_CVT \
    FXP_MIX("%[v3]", "%[w6]", "0") FXP_RL("%[n6]", L6) FXP_CVT FXP_MIX("%[v3]", "%[w7]", "1") FXP_RL("%[n7]", L7) FXP_CVT
// the slow key (fx_key_slow): the sign of w selects ms = -w, vs = 1 or ms = 1,
// vs = w; w is copied to a VGPR first (one SGPR operand per VALU instruction
// besides vcc)
#define FXP_SLOW1(VI, W, SEL, N, L)                                              \
    "v_mov_b32 %[x], " W "\n\t"                                                   \
    "v_cmp_gt_i32 vcc, 0, %[x]\n\t"                                               \
    "v_cndmask_b32_e64 %[ms], 1.0, -%[x], vcc\n\t"                                \
    "v_cndmask_b32_e64 %[vs], %[x], 1.0, vcc\n\t"                                 \
    "v_cvt_f32_f16 %[t], %[a]\n\t"                                                \
    FXP_RL(N, L)                                                                  \
    "v_mul_f32 %[t], %[t], %[ms]\n\t"                                             \
    "v_cvt_f16_f32 %[a], %[t]\n\t"                                                \
    "v_fma_mix_f32 %[t], " VI ", %[vs], %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t" \
    "v_cvt_f16_f32 %[a], %[t]\n\t"
#define FXP_SLOW_BODY(L0, L1, L2, L3, L4, L5, L6, L7)                                                                   \
    FXP_SLOW1("%[v0]", "%[w0]", "0", "%[n0]", L0) FXP_SLOW1("%[v0]", "%[w1]", "1", "%[n1]", L1)                          \
    FXP_SLOW1("%[v1]", "%[w2]", "0", "%[n2]", L2) FXP_SLOW1("%[v1]", "%[w3]", "1", "%[n3]", L3)                          \
    FXP_SLOW1("%[v2]", "%[w4]", "0", "%[n4]", L4) FXP_SLOW1("%[v2]", "%[w5]", "1", "%[n5]", L5)                          \
    FXP_SLOW1("%[v3]", "%[w6]", "0", "%[n6]", L6) FXP_SLOW1("%[v3]", "%[w7]", "1", "%[n7]", L7)
#define FXP_OUTS [t] "=&v"(t), [a] "+v"(acc), [n0] "=&s"(n[0]), [n1] "=&s"(n[1]), [n2] "=&s"(n[2]), [n3] "=&s"(n[3]), \
                 [n4] "=&s"(n[4]), [n5] "=&s"(n[5]), [n6] "=&s"(n[6]), [n7] "=&s"(n[7])
#define FXP_INS [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(w[0]), [w1] "s"(w[1]), [w2] "s"(w[2]), \
                [w3] "s"(w[3]), [w4] "s"(w[4]), [w5] "s"(w[5]), [w6] "s"(w[6]), [w7] "s"(w[7]), [wn] "v"(wn)

// the checked form, for buffers holding a new maximum: per key one SALU test
// of the key's bit in m64 (uniform) and a branch out of line only for a
// record key (scale by ms = -w, then add v * 1: fx_key_slow), so the other
// keys of its 8-key group keep the two-instruction step
#define FXP_CHK1(VI, W, SEL, N, L, B)                                                            \
    "v_readlane_b32 " N ", %[wn], " #L "\n\t"                                                  \
    "s_bitcmp1_b64 %[m], " #B "\n\t"                                                          \
    "s_cbranch_scc1 Lr" #B "_%=\n\t"                                                     \
    "v_fma_mix_f32 %[t], " VI ", " W ", %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"       \
    "v_cvt_f16_f32 %[a], %[t]\n"                                                               \
    "Lb" #B "_%=:\n\t"
#define FXP_REC1(VI, W, SEL, B)                                                                  \
    "Lr" #B "_%=:\n\t"                                                                   \
    "v_cvt_f32_f16 %[t], %[a]\n\t"                                                            \
    "v_mul_f32_e64 %[t], -" W ", %[t]\n\t"                                                    \
    "v_cvt_f16_f32 %[a], %[t]\n\t"                                                            \
    "v_fma_mix_f32 %[t], " VI ", 1.0, %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"        \
    "v_cvt_f16_f32 %[a], %[t]\n\t"                                                            \
    "s_branch Lb" #B "_%=\n\t"
template <int LN, int G>
__device__ __forceinline__ void fxp8_chk(f16 &acc, const u32x4 v, const int (&w)[8], float wn, int (&n)[8], unsigned long long m);

template <int LN>
__device__ __forceinline__ void fxp8_fast(f16 &acc, const u32x4 v, const int (&w)[8], float wn, int (&n)[8]);
template <int LN>
__device__ __forceinline__ void fxp8_slow(f16 &acc, const u32x4 v, const int (&w)[8], float wn, int (&n)[8]);

#define FXP_DEF(LN, L0, L1, L2, L3, L4, L5, L6, L7)                                                               \
    template <>                                                                                                   \
    __device__ __forceinline__ void fxp8_fast<LN>(f16 & acc, const u32x4 v, const int(&w)[8], float wn, int(&n)[8]) { \
        float t;                                                                                                  \
        asm volatile(FXP_FAST_BODY(L0, L1, L2, L3, L4, L5, L6, L7) : FXP_OUTS : FXP_INS);                         \
    }                                                                                                             \
    template <>                                                                                                   \
    __device__ __forceinline__ void fxp8_slow<LN>(f16 & acc, const u32x4 v, const int(&w)[8], float wn, int(&n)[8]) { \
        float t, x, ms, vs;                                                                                       \
        asm volatile(FXP_SLOW_BODY(L0, L1, L2, L3, L4, L5, L6, L7)                                                 \
                     : FXP_OUTS, [x] "=&v"(x), [ms] "=&v"(ms), [vs] "=&v"(vs) : FXP_INS : "vcc");              \
    }
#define FXP_CHK_DEF(LN, G, L0, L1, L2, L3, L4, L5, L6, L7, B0, B1, B2, B3, B4, B5, B6, B7)                              \
    template <>                                                                                                      \
    __device__ __forceinline__ void fxp8_chk<LN, G>(f16 & acc, const u32x4 v, const int(&w)[8], float wn, int(&n)[8],   \
                                                     unsigned long long m) {                                         \
        float t;                                                                                                     \
        asm volatile(FXP_CHK1("%[v0]", "%[w0]", "0", "%[n0]", L0, B0) FXP_CHK1("%[v0]", "%[w1]", "1", "%[n1]", L1, B1)   \
                     FXP_CHK1("%[v1]", "%[w2]", "0", "%[n2]", L2, B2) FXP_CHK1("%[v1]", "%[w3]", "1", "%[n3]", L3, B3)   \
                     FXP_CHK1("%[v2]", "%[w4]", "0", "%[n4]", L4, B4) FXP_CHK1("%[v2]", "%[w5]", "1", "%[n5]", L5, B5)   \
                     FXP_CHK1("%[v3]", "%[w6]", "0", "%[n6]", L6, B6) FXP_CHK1("%[v3]", "%[w7]", "1", "%[n7]", L7, B7)   \
                     "s_branch Le_%=\n\t"                                                                      \
                     FXP_REC1("%[v0]", "%[w0]", "0", B0) FXP_REC1("%[v0]", "%[w1]", "1", B1)                          \
                     FXP_REC1("%[v1]", "%[w2]", "0", B2) FXP_REC1("%[v1]", "%[w3]", "1", B3)                          \
                     FXP_REC1("%[v2]", "%[w4]", "0", B4) FXP_REC1("%[v2]", "%[w5]", "1", B5)                          \
                     FXP_REC1("%[v3]", "%[w6]", "0", B6) FXP_REC1("%[v3]", "%[w7]", "1", B7)                          \
                     "Le_%=:"                                                                                  \
                     : FXP_OUTS : FXP_INS, [m] "s"(m) : "scc");                                                     \
    }
FXP_CHK_DEF(8, 0, 8, 9, 10, 11, 12, 13, 14, 15, 0, 1, 2, 3, 4, 5, 6, 7)
FXP_CHK_DEF(16, 1, 16, 17, 18, 19, 20, 21, 22, 23, 8, 9, 10, 11, 12, 13, 14, 15)
FXP_CHK_DEF(24, 2, 24, 25, 26, 27, 28, 29, 30, 31, 16, 17, 18, 19, 20, 21, 22, 23)
FXP_CHK_DEF(32, 3, 32, 33, 34, 35, 36, 37, 38, 39, 24, 25, 26, 27, 28, 29, 30, 31)
FXP_CHK_DEF(40, 4, 40, 41, 42, 43, 44, 45, 46, 47, 32, 33, 34, 35, 36, 37, 38, 39)
FXP_CHK_DEF(48, 5, 48, 49, 50, 51, 52, 53, 54, 55, 40, 41, 42, 43, 44, 45, 46, 47)
FXP_CHK_DEF(56, 6, 56, 57, 58, 59, 60, 61, 62, 63, 48, 49, 50, 51, 52, 53, 54, 55)
FXP_CHK_DEF(0, 7, 0, 1, 2, 3, 4, 5, 6, 7, 56, 57, 58, 59, 60, 61, 62, 63)
#undef FXP_CHK_DEF
#undef FXP_CHK1
#undef FXP_REC1
FXP_DEF(0, 0, 1, 2, 3, 4, 5, 6, 7)
FXP_DEF(8, 8, 9, 10, 11, 12, 13, 14, 15)
FXP_DEF(16, 16, 17, 18, 19, 20, 21, 22, 23)
FXP_DEF(24, 24, 25, 26, 27, 28, 29, 30, 31)
FXP_DEF(32, 32, 33, 34, 35, 36, 37, 38, 39)
FXP_DEF(40, 40, 41, 42, 43, 44, 45, 46, 47)
FXP_DEF(48, 48, 49, 50, 51, 52, 53, 54, 55)
FXP_DEF(56, 56, 57, 58, 59, 60, 61, 62, 63)
#undef FXP_DEF
#undef FXP_MIX
#undef FXP_RL
#undef FXP_CVT
#undef FXP_FAST_BODY
#undef FXP_SLOW1
#undef FXP_SLOW_BODY
#undef FXP_OUTS
#undef FXP_INS

// group G of a buffer (keys 8 G .. 8 G + 7): its weights w (SGPRs) in, the
// next group's out (lanes 8 G + 8 .. of wc, or lanes 0 .. 7 of wnb, the next
// buffer's weights, after the last group)
template <int G>
__device__ __forceinline__ void fxp_group(f16 &acc, const u32x4 v, int (&w)[8], float wc, float wnb, unsigned long long m64) {
    int n[8];
#ifdef FXP_CHK   // per-key test and out-of-line record keys: measured slower (the blocks' code size)
    if (m64 != 0) {   // (a compile-time 0 in the fast buffer: no test)
        if constexpr (G < 7) fxp8_chk<8 * G + 8, G>(acc, v, w, wc, n, m64);
        else fxp8_chk<0, 7>(acc, v, w, wnb, n, m64);
    } else
#else
    if (((m64 >> (8 * G)) & 0xffull) != 0) {   // a group holding a new maximum: every key on the slow block
        if constexpr (G < 7) fxp8_slow<8 * G + 8>(acc, v, w, wc, n);
        else fxp8_slow<0>(acc, v, w, wnb, n);
    } else
#endif
    {
        if constexpr (G < 7) fxp8_fast<8 * G + 8>(acc, v, w, wc, n);
        else fxp8_fast<0>(acc, v, w, wnb, n);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = n[i];
}

// the 64 keys of one buffer: v = their V (8 keys per u32x4), w = group 0's
// weights in SGPRs on entry, the next buffer's group 0 on exit; wc = this
// buffer's weights (lane = key), wnb = the next buffer's, m64 = this
// buffer's new-maximum bits (uniform).  One branch per buffer: a buffer
// without a maximum runs 8 straight fast groups.
__device__ __forceinline__ void fxp_buffer(f16 &acc, const u32x4 *v, int (&w)[8], float wc, float wnb, unsigned long long m64) {
#ifdef FXP_NO_CHK   // (timing experiments only: every buffer on the fast blocks, wrong where a key is a new maximum)
    m64 = 0ull;
#endif
    if (__builtin_expect(m64 != 0ull, 0)) {
        fxp_group<0>(acc, v[0], w, wc, wnb, m64);
        fxp_group<1>(acc, v[1], w, wc, wnb, m64);
        fxp_group<2>(acc, v[2], w, wc, wnb, m64);
        fxp_group<3>(acc, v[3], w, wc, wnb, m64);
        fxp_group<4>(acc, v[4], w, wc, wnb, m64);
        fxp_group<5>(acc, v[5], w, wc, wnb, m64);
        fxp_group<6>(acc, v[6], w, wc, wnb, m64);
        fxp_group<7>(acc, v[7], w, wc, wnb, m64);
    } else {
        fxp_group<0>(acc, v[0], w, wc, wnb, 0ull);
        fxp_group<1>(acc, v[1], w, wc, wnb, 0ull);
        fxp_group<2>(acc, v[2], w, wc, wnb, 0ull);
        fxp_group<3>(acc, v[3], w, wc, wnb, 0ull);
        fxp_group<4>(acc, v[4], w, wc, wnb, 0ull);
        fxp_group<5>(acc, v[5], w, wc, wnb, 0ull);
        fxp_group<6>(acc, v[6], w, wc, wnb, 0ull);
        fxp_group<7>(acc, v[7], w, wc, wnb, 0ull);
    }
}

// group 0's weights of a buffer into SGPRs
__device__ __forceinline__ void fxp_first(float wc, int (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wc), i);
}

// The whole chain of one (head, row) for this wave's 64 dimensions: keys
// [0, nl) through the loop, V from the V^T cache (vt: the wave's key block 0,
// loff = 8 lane; blocks past lastb re-read it, fx_loadQ).  Scores from src:
// p = src.issue(j0) requests this lane's key j0 + lane, src.take(p, j0)
// returns it (-inf at and past n; it may poll) -- issued a buffer and a half
// before they are needed.  Keys nl .. n - 1 (the fused launch's new key: at
// most one) are scored and counted in M and S but not accumulated: the loop
// sees weight 0 there and the key's weight is returned in wlast for the
// caller to apply (fx_key_slow).  Returns S (summed over the wave).
// FXP_TRACE (tools/micro/chain_pipe.hip only): per-phase shader cycles of
// wave 0 of workgroup 0 -- [weights, chain] summed over the buffers
#ifdef FXP_TRACE
__device__ unsigned long long fxp_trace[4];
#define FXP_T0() const unsigned long long _ft0 = __builtin_readcyclecounter()
#define FXP_T1(i) do { if (blockIdx.x == 0 && threadIdx.x == 0) fxp_trace[i] += __builtin_readcyclecounter() - _ft0; } while (0)
#else
#define FXP_T0()
#define FXP_T1(i)
#endif
template <class Src>
__device__ __forceinline__ float fxp_chain(const Src &src, const uint16_t *__restrict__ vt, int loff, int nl, int lastb, f16 &acc,
                                           float &wlast) {
    const int lane = threadIdx.x & 63;
    float M = -INFINITY, Sl = 0.0f, wl = 0.0f;
    auto wts = [&](float s, int j0, unsigned long long &m) {
        float x = fxp_weights(s, M, Sl, m);
        if (j0 + 64 > nl) {   // (weights past the loop keys: 0, their maximum bits cleared; key nl saved)
            const int j = j0 + lane;
            if (j == nl) wl = x;
            if (j >= nl) x = 0.0f;
            m &= nl - j0 <= 0 ? 0ull : (1ull << (nl - j0)) - 1ull;
        }
        return x;
    };
    unsigned long long m0, m1;
    u32x4 va[DX_Q / 8], vb[DX_Q / 8];
    // (vt and lastb are wave-uniform; readfirstlane says so, else every load
    // becomes a waterfall loop over the lanes' descriptors)
    const unsigned long long vtu = (unsigned long long)vt;
    const uint16_t *vts = (const uint16_t *)(((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(vtu >> 32)) << 32) |
                                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)vtu));
    lastb = __builtin_amdgcn_readfirstlane(lastb);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)vts, (short)0, (lastb + 1) * 2048, 0x00020000);
    const int voff = 2 * loff;
    fxp_loadQ(va, rs, voff, 0, lastb);
    auto q0 = src.issue(0);
    auto q1 = src.issue(DX_Q);
    auto q2 = src.issue(2 * DX_Q);
    float wa = wts(src.take(q0, 0), 0, m0), wb;
    int w[8];
    fxp_first(wa, w);
    for (int j0 = 0; j0 < nl; j0 += 2 * DX_Q) {
        fxp_loadQ(vb, rs, voff, j0 + DX_Q, lastb);
        {
            FXP_T0();
            wb = wts(src.take(q1, j0 + DX_Q), j0 + DX_Q, m1);
            FXP_T1(0);
        }
        q1 = src.issue(j0 + 3 * DX_Q);
        {
            FXP_T0();
            fxp_buffer(acc, va, w, wa, wb, m0);
            FXP_T1(1);
        }
        if (j0 + DX_Q >= nl) break;
        fxp_loadQ(va, rs, voff, j0 + 2 * DX_Q, lastb);
        {
            FXP_T0();
            wa = wts(src.take(q2, j0 + 2 * DX_Q), j0 + 2 * DX_Q, m0);
            FXP_T1(0);
        }
        q2 = src.issue(j0 + 4 * DX_Q);
        {
            FXP_T0();
            fxp_buffer(acc, vb, w, wb, wa, m1);
            FXP_T1(1);
        }
    }
    wlast = lane_f(wl, nl & 63);
    return wave_sum(Sl);
}

// fxp_chain with the weights given (the splits computed them, attention.hip
// split_weights): src.take returns key j0 + lane's signed weight (0 at and past
// n); a buffer's new-maximum bits are the sign bits.  Same chain, same handling
// of keys nl .. n - 1 (weight 0 in the loop, key nl's weight in wlast).
//
// V^T through a ring of 8 two-group slots (16 keys, 64 VGPRs as fxp_chain's
// two 64-key buffers): a slot is reloaded with the keys 128 ahead as soon as
// its two groups are done, so each load has 112 keys of chain time (~1.7k
// cycles) to land instead of 64: in the fused launch the V^T rows come from
// the XCD's L2 under the o-projection's weight stream, and with one buffer of
// lead the chain waited on them (~5 cycles a key, device trace with every load
// cache-hot: 20.4 -> 15.3).
template <int S>   // reload ring slot S (groups 2S, 2S + 1) with the key blocks at jb, jb + 1
__device__ __forceinline__ void fxp_ring_load(u32x4 (&r)[16], __amdgpu_buffer_rsrc_t rs, int voff, int jb, int lastb) {
    r[2 * S] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, min(jb, lastb) * 2048, 0));
    r[2 * S + 1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, min(jb + 1, lastb) * 2048, 0));
}
// the 64 keys of ring half H (groups 8H .. 8H + 7, keys from jk), reloading
// each slot with the keys 128 ahead once its groups are done; one branch on
// m64 (a buffer without a new maximum: straight fast groups)
template <int H, bool SLOWOK>
__device__ __forceinline__ void fxp_ring_body(f16 &acc, u32x4 (&r)[16], int (&w)[8], float wc, float wnb, unsigned long long m64,
                                              __amdgpu_buffer_rsrc_t rs, int voff, int jk, int lastb) {
    const int jb = (jk + 128) / 8;   // the key block the half's first slot reloads
    fxp_group<0>(acc, r[8 * H + 0], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_group<1>(acc, r[8 * H + 1], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_ring_load<4 * H + 0>(r, rs, voff, jb, lastb);
    fxp_group<2>(acc, r[8 * H + 2], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_group<3>(acc, r[8 * H + 3], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_ring_load<4 * H + 1>(r, rs, voff, jb + 2, lastb);
    fxp_group<4>(acc, r[8 * H + 4], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_group<5>(acc, r[8 * H + 5], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_ring_load<4 * H + 2>(r, rs, voff, jb + 4, lastb);
    fxp_group<6>(acc, r[8 * H + 6], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_group<7>(acc, r[8 * H + 7], w, wc, wnb, SLOWOK ? m64 : 0ull);
    fxp_ring_load<4 * H + 3>(r, rs, voff, jb + 6, lastb);
}
template <int H>
__device__ __forceinline__ void fxp_ring_half(f16 &acc, u32x4 (&r)[16], int (&w)[8], float wc, float wnb, unsigned long long m64,
                                              __amdgpu_buffer_rsrc_t rs, int voff, int jk, int lastb) {
#ifdef FXP_NO_CHK   // (timing experiments only)
    m64 = 0ull;
#endif
    if (__builtin_expect(m64 != 0ull, 0)) fxp_ring_body<H, true>(acc, r, w, wc, wnb, m64, rs, voff, jk, lastb);
    else fxp_ring_body<H, false>(acc, r, w, wc, wnb, 0ull, rs, voff, jk, lastb);
}
template <class Src>
__device__ __forceinline__ void fxp_chain_w(const Src &src, const uint16_t *__restrict__ vt, int loff, int nl, int lastb, f16 &acc,
                                            float &wlast) {
    const int lane = threadIdx.x & 63;
    float wl = 0.0f;
    auto wts = [&](float x, int j0, unsigned long long &m) {
        if (j0 + 64 > nl) {
            const int j = j0 + lane;
            if (j == nl) wl = x;
            if (j >= nl) x = 0.0f;
        }
        m = __ballot(__builtin_signbit(x));
        return x;
    };
    unsigned long long m0, m1;
    const unsigned long long vtu = (unsigned long long)vt;
    const uint16_t *vts = (const uint16_t *)(((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(vtu >> 32)) << 32) |
                                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)vtu));
    lastb = __builtin_amdgcn_readfirstlane(lastb);
#ifdef FXP_HOTV   // (timing experiments only: every V^T load reads key block 0)
    lastb = 0;
#endif
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)vts, (short)0, (lastb + 1) * 2048, 0x00020000);
    const int voff = 2 * loff;
    u32x4 r[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
        r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, min(i, lastb) * 2048, 0));
    auto q0 = src.issue(0);
    auto q1 = src.issue(DX_Q);
    auto q2 = src.issue(2 * DX_Q);
    float wa = wts(src.take(q0, 0), 0, m0), wb;
    int w[8];
    fxp_first(wa, w);
    for (int j0 = 0; j0 < nl; j0 += 2 * DX_Q) {
        wb = wts(src.take(q1, j0 + DX_Q), j0 + DX_Q, m1);
        q1 = src.issue(j0 + 3 * DX_Q);
        fxp_ring_half<0>(acc, r, w, wa, wb, m0, rs, voff, j0, lastb);
        if (j0 + DX_Q >= nl) break;
        wa = wts(src.take(q2, j0 + 2 * DX_Q), j0 + 2 * DX_Q, m0);
        q2 = src.issue(j0 + 4 * DX_Q);
        fxp_ring_half<1>(acc, r, w, wb, wa, m1, rs, voff, j0 + DX_Q, lastb);
    }
    wlast = lane_f(wl, nl & 63);
}

// scores from memory (global or LDS), one float per key
struct FxpScores {
    const float *sc;
    int n;
    __device__ __forceinline__ float issue(int j0) const {
        const int j = j0 + (int)(threadIdx.x & 63);
        return sc[j < n ? j : 0];
    }
    __device__ __forceinline__ float take(float v, int j0) const { return j0 + (int)(threadIdx.x & 63) < n ? v : -INFINITY; }
};

}  // namespace qasr
