// fx_chain.h -- the decode-step chain of ggml's CPU flash attention, shared by
// the separate exact decode kernels (fa_exact.hip) and the batch-1 fused
// launch (attention.hip qkv_attn1_kernel, chain role).
//
// ggml_flash_attn_ext on the CPU backend (src/text_decoder.cpp:534-540;
// SURVEY.md §8(a) viii) walks one query row's keys in order: s = q.k * scale;
// a new maximum rescales the fp16 V accumulator (ggml_vec_scale_f16: y =
// fp16(fp32(y) * ms)), every key adds v * vs (ggml_vec_mad_f16: y =
// fp16(fma(fp32(v), vs, fp32(y)))), and S = S * ms + vs in fp32.  Each
// (query, head, dimension) is one sequential chain; here one dimension a lane,
// V from the V^T cache (kernels.h vt_index: 8 keys of a dimension per 16-B
// load), the key's weight an SGPR operand (v_readlane) of v_fma_mix_f32.
//
// Weights are kept one register per key: w = vs where the key is not a new
// maximum, w = -ms where it is (vs = 1 there; ms in [0, 1), the first key's
// ms = exp(-inf) = 0 is stored as -0.0f) -- the sign bit tells the two apart,
// so a chunk's weights cost 32 VGPRs instead of 64.
#pragma once
#include "dev_common.h"

namespace qasr {

#define DX_B 32    // keys per lane of the weights = keys sharing one fast/slow decision
#define DX_Q 64    // keys of V per register buffer (two in turn)
#define DX_KC (64 * DX_B)   // keys per weights chunk (one wave: 64 lanes x DX_B)

// one value: the conversion in asm (a scalar fptrunc of an fma would fold
// into v_fma_mixlo_f16, which rounds once instead of fp32-then-fp16)
__device__ __forceinline__ f16 fx_cvt(float f) {
    f16 h;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(h) : "v"(f));
    return h;
}
// ggml_vec_mad_f16 on one value: fp16(fma(v, vs, acc)), the fma rounded to fp32
__device__ __forceinline__ f16 fx_mad1(f16 acc, uint16_t v, float vs) {
    return fx_cvt(fmaf((float)__builtin_bit_cast(f16, v), vs, (float)acc));
}

// DPP lane move with -inf where the source lane is out of range or its row
// is masked off (bound_ctrl off: the lane keeps the -inf of `old`)
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_ninf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, -INFINITY), __builtin_bit_cast(int, v),
                                                                 CTRL, ROWS, 0xF, false));
}
// inclusive prefix maximum over the 64 lanes, all in VALU DPP: Hillis-Steele
// in each 16-lane row (row_shr 1, 2, 4, 8), then row_bcast:15 (each row's
// last lane into the next row) and row_bcast:31 (lane 31 into rows 2, 3)
__device__ __forceinline__ float wave_scan_max(float x) {
    x = fmaxf(x, dpp_ninf<0x111, 0xF>(x));
    x = fmaxf(x, dpp_ninf<0x112, 0xF>(x));
    x = fmaxf(x, dpp_ninf<0x114, 0xF>(x));
    x = fmaxf(x, dpp_ninf<0x118, 0xF>(x));
    x = fmaxf(x, dpp_ninf<0x142, 0xA>(x));
    x = fmaxf(x, dpp_ninf<0x143, 0xC>(x));
    return x;
}

__device__ __forceinline__ uint16_t fx_elem(const u32x4 *v, int i) {   // key i of the buffer (i constant)
    const uint32_t w = v[i >> 3][(i >> 1) & 3];
    return (uint16_t)((i & 1) ? (w >> 16) : (w & 0xffffu));
}
__device__ __forceinline__ float fx_lane(float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
// one key of the slow path, branch-free: w signed as above (uniform), so
// ms = 1 and vs = w, or ms = -w and vs = 1 -- the scale is exact where ms = 1
// (an fp16 value times 1), and a zero weight (keys past the chunk) leaves the
// accumulator unchanged (fma(v, 0, acc) = acc for finite v)
__device__ __forceinline__ f16 fx_key_slow(f16 acc, uint16_t v, float w) {
    const bool nm = __builtin_signbit(w);
    acc = fx_cvt((float)acc * (nm ? -w : 1.0f));
    return fx_mad1(acc, v, nm ? 1.0f : w);
}

// keys [j0, min(j0 + DX_Q, n)) of the chunk (relative to its first key) from
// registers v, in 32-key batches, one dimension a lane (the decode chains of
// fx_decode.h).  w: the weights registers (key 32 L + i in lane L, element i;
// zero past the chunk's keys); flags: bit L = lane L's batch holds a new
// maximum or keys past the chunk -- the others take two VALU instructions a
// key.  In a flagged batch the slow path is decided per 8-key group:
// kb = this lane's new-maximum bits (bit i: key 32 lane + i, fx_weights_reg),
// read for batch L by v_readlane; groups without a maximum take the fast path
// (keys past n carry zero weights: exact no-ops there)
__device__ __forceinline__ void fx_step1_m(const u32x4 *v, int j0, int n, const float *w, unsigned long long flags, uint32_t kb,
                                           f16 &acc) {
#pragma unroll
    for (int bq = 0; bq < DX_Q / DX_B; bq++) {
        const int jb = j0 + bq * DX_B;
        const int L = jb / DX_B;
        if (jb >= n) break;
        if (!((flags >> L) & 1ull)) {
#pragma unroll
            for (int i = 0; i < DX_B; i++) acc = fx_mad1(acc, fx_elem(v, bq * DX_B + i), fx_lane(w[i], L));
        } else {
            const uint32_t m32 = (uint32_t)__builtin_amdgcn_readlane((int)kb, L);
#pragma unroll
            for (int g = 0; g < DX_B / 8; g++) {
                if ((m32 >> (8 * g)) & 0xffu) {
#pragma unroll
                    for (int i = 8 * g; i < 8 * g + 8; i++) acc = fx_key_slow(acc, fx_elem(v, bq * DX_B + i), fx_lane(w[i], L));
                } else {
#pragma unroll
                    for (int i = 8 * g; i < 8 * g + 8; i++) acc = fx_mad1(acc, fx_elem(v, bq * DX_B + i), fx_lane(w[i], L));
                }
            }
        }
    }
}
// fx_step1_m with the weights in LDS instead of registers (the fused launch's
// chain role): ws = the head's signed weights, FX_ST floats per 32-key row
// (row L = lane L's keys of fx_weights_reg).  Per 8 keys the weights arrive
// as two uniform ds_read_b128 (VGPR operands of v_fma_mix_f32), requested one
// group ahead; the fast path of a group is one inline-asm block of the
// chain's 16 instructions -- the compiler neither hoists the next groups'
// loads above it (the "memory" clobber) nor interleaves anything into it, so
// the role's register use stays bounded (compiler-scheduled, the unrolled
// 64-key step held up to 190 VGPRs).  The arithmetic is fx_mad1's:
// v_fma_mix_f32 (fp16 v and accumulator, fp32 weight, one fp32 rounding),
// then v_cvt_f16_f32 (RNE).
#define FX_ST 36   // LDS floats per 32-key row: the 64 rows' 16-B reads of fx_weights_reg hit distinct banks
#define FX_MIX(VI, W, SEL) "v_fma_mix_f32 %0, " VI ", " W ", %1 op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
// (no wait state between the mix and the convert: the hardware interlocks the
// dependency; tools/micro/chain_asm.hip: bit-identical, 13.1 cycles a key
// against 17.1 with an s_nop 0 -- the padding hipcc adds in front of an asm
// statement that reads a just-written VGPR)
#define FX_CVT "v_cvt_f16_f32 %1, %0\n\t"
__device__ __forceinline__ void fx8_fast(f16 &acc, const u32x4 v, const floatx4 wa, const floatx4 wb) {
    float t;
    asm volatile(FX_MIX("%2", "%6", "0") FX_CVT FX_MIX("%2", "%7", "1") FX_CVT FX_MIX("%3", "%8", "0") FX_CVT
                 FX_MIX("%3", "%9", "1") FX_CVT FX_MIX("%4", "%10", "0") FX_CVT FX_MIX("%4", "%11", "1") FX_CVT
                 FX_MIX("%5", "%12", "0") FX_CVT FX_MIX("%5", "%13", "1") FX_CVT
                 : "=&v"(t), "+v"(acc)
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(wa[0]), "v"(wa[1]), "v"(wa[2]), "v"(wa[3]), "v"(wb[0]),
                   "v"(wb[1]), "v"(wb[2]), "v"(wb[3])
                 : "memory");
}
#undef FX_MIX
#undef FX_CVT
// the slow path of 8 keys as one asm block too (fx_key_slow's arithmetic:
// the sign of w selects ms = -w, vs = 1 or ms = 1, vs = w; the scale is
// fp16(fp32(acc) * ms), exact where ms = 1), so the chain loop stays a few
// hundred bytes of straight code per group -- with the slow path as compiler
// code between the fast blocks the fused launch's chain ran 21 us instead of
// 12 at 1.37k keys (device trace; instruction fetch over ~30 KB of loop)
#define FX_SLOW1(VI, W, SEL)                                                   \
    "v_cmp_gt_i32 vcc, 0, " W "\n\t"                                         \
    "v_cndmask_b32_e64 %2, 1.0, -" W ", vcc\n\t"                              \
    "v_cndmask_b32_e64 %3, " W ", 1.0, vcc\n\t"                               \
    "v_cvt_f32_f16 %0, %1\n\t"                                                \
    "v_mul_f32 %0, %0, %2\n\t"                                                \
    "v_cvt_f16_f32 %1, %0\n\t"                                                \
    "v_fma_mix_f32 %0, " VI ", %3, %1 op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t" \
    "v_cvt_f16_f32 %1, %0\n\t"
__device__ __forceinline__ void fx8_slow(f16 &acc, const u32x4 v, const floatx4 wa, const floatx4 wb) {
    float t, ms, vs;
    asm volatile(FX_SLOW1("%4", "%8", "0") FX_SLOW1("%4", "%9", "1") FX_SLOW1("%5", "%10", "0") FX_SLOW1("%5", "%11", "1")
                 FX_SLOW1("%6", "%12", "0") FX_SLOW1("%6", "%13", "1") FX_SLOW1("%7", "%14", "0") FX_SLOW1("%7", "%15", "1")
                 : "=&v"(t), "+v"(acc), "=&v"(ms), "=&v"(vs)
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(wa[0]), "v"(wa[1]), "v"(wa[2]), "v"(wa[3]), "v"(wb[0]),
                   "v"(wb[1]), "v"(wb[2]), "v"(wb[3])
                 : "vcc", "memory");
}
#undef FX_SLOW1
__device__ __forceinline__ void fx_w8(const float *ws, int k, floatx4 &wa, floatx4 &wb) {   // weights of keys k .. k + 7
    const float *p = ws + (k >> 5) * FX_ST + (k & 31);
    wa = *(const floatx4 *)p;
    wb = *(const floatx4 *)(p + 4);
}
// keys [j0, j0 + DX_Q) from registers v (8 keys per u32x4); every weight past
// the keys to take is 0 in ws (a no-op: fma(v, 0, acc) = acc).  wa / wb: the
// weights of keys j0 .. j0 + 7 on entry, of j0 + DX_Q .. on exit.  One
// decision per 64 keys: both 32-key batches fast (the common case: one
// straight 1 KiB block, no branch inside), else all 64 keys on the slow path
// -- exact for every key (ms = 1 leaves the accumulator unchanged), placed out
// of line.  Branching per 8-key group cost ~2x in the fused launch (a taken
// branch and an instruction fetch every 16 instructions; device trace).
__device__ __forceinline__ void fx_step1_lds(const u32x4 *v, int j0, const float *ws, unsigned long long flags, f16 &acc,
                                             floatx4 &wa, floatx4 &wb) {
    if (__builtin_expect(((flags >> (j0 / DX_B)) & 3ull) != 0, 0)) {
#pragma unroll
        for (int g8 = 0; g8 < DX_Q / 8; g8++) {
            floatx4 na, nb;
            fx_w8(ws, j0 + 8 * g8 + 8, na, nb);   // (row padding / the next row: in bounds of the chunk's LDS image)
            fx8_slow(acc, v[g8], wa, wb);
            wa = na;
            wb = nb;
        }
    } else {
#pragma unroll
        for (int g8 = 0; g8 < DX_Q / 8; g8++) {
            floatx4 na, nb;
            fx_w8(ws, j0 + 8 * g8 + 8, na, nb);
            fx8_fast(acc, v[g8], wa, wb);
            wa = na;
            wb = nb;
        }
    }
}

// fx_step1_lds with the slow path taken per 8-key group: m64 (uniform, in
// SGPRs) = the 64 keys' new-maximum bits, bit i for key j0 + i.  A buffer
// without a maximum runs the straight fast block (one branch per 64 keys);
// one with a maximum decides per 8-key group, so only the groups holding one
// run the slow asm block (per-group branches in every buffer measured 16 us a
// chain against 13: a branch pair per 16 instructions); keys past the chunk
// carry zero weights, which the fast path leaves as exact no-ops
// (fma(v, 0, acc) = acc).  A running maximum over
// n random scores has ~ln n records, so per-64-key decisions sent ~6 of 22
// buffers of a 1.37k-key chain down the slow path.
__device__ __forceinline__ void fx_step1_lds_m(const u32x4 *v, int j0, const float *ws, unsigned long long m64, f16 &acc,
                                               floatx4 &wa, floatx4 &wb) {
    if (__builtin_expect(m64 != 0ull, 0)) {   // out of line: per-group decisions only in a buffer holding a maximum
#pragma unroll
        for (int g8 = 0; g8 < DX_Q / 8; g8++) {
            floatx4 na, nb;
            fx_w8(ws, j0 + 8 * g8 + 8, na, nb);
            if (((m64 >> (8 * g8)) & 0xffull) != 0) fx8_slow(acc, v[g8], wa, wb);
            else fx8_fast(acc, v[g8], wa, wb);
            wa = na;
            wb = nb;
        }
    } else {
#pragma unroll
        for (int g8 = 0; g8 < DX_Q / 8; g8++) {
            floatx4 na, nb;
            fx_w8(ws, j0 + 8 * g8 + 8, na, nb);
            fx8_fast(acc, v[g8], wa, wb);
            wa = na;
            wb = nb;
        }
    }
}
// the 64 new-maximum bits of keys j0 .. j0 + 63 from km (u16 per 16 keys) as a
// uniform value
__device__ __forceinline__ unsigned long long fx_mask64(const uint16_t *km, int j0) {
    const uint2 m = *(const uint2 *)(km + j0 / 16);
    return ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)m.y) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)m.x);
}

// DX_Q keys of V from key block j0 / 8 (vt: the wave's key block 0, uniform;
// loff = 8 lane: kernels.h vt_index, 1024 halves per block).  Blocks past
// lastb (the sequence's last key block, uniform) re-read block lastb: the
// loads still issue, so the callers' wait counts stay exact, but the
// read-ahead past the context hits the cache instead of streaming up to two
// steps of unused V^T from HBM (~30 % of a 64 x 30 s batch's V^T traffic).
__device__ __forceinline__ void fx_loadQ(u32x4 *v, const uint16_t *__restrict__ vt, int loff, int j0, int lastb = 1 << 28) {
#pragma unroll
    for (int i = 0; i < DX_Q / 8; i++) v[i] = *(const u32x4 *)(vt + (long)min(j0 / 8 + i, lastb) * 1024 + loff);
}

// The weights of a chunk's n keys (n <= DX_KC) for one wave, in registers:
// lane L's keys 32 L + i -> w[i] (signed as above; 0 past n); flags bit L =
// lane L's batch takes the slow path (fx_step1).  src(j) = the scaled score of key j (-inf: masked, vs =
// 0, ms = 1).  M: running maximum (in/out).  Returns this chunk's S at the new
// maximum (per lane a sequential S = S * ms + vs as ggml, the lanes combined
// in fp32).  wlast: the weight of key n - 1 (uniform).
template <class Src>
__device__ __forceinline__ float fx_weights_reg(Src src, int n, float &M, float *w, unsigned long long &flags, float &wlast,
                                                uint32_t *kbits = nullptr) {
    const int lane = threadIdx.x & 63;
    float lm = -INFINITY;
#pragma unroll
    for (int i = 0; i < DX_B; i++) {
        const int j = lane * DX_B + i;
        w[i] = j < n ? src(j) : -INFINITY;   // the score, replaced by the weight below
    }
#pragma unroll
    for (int i = 0; i < DX_B; i++) lm = fmaxf(lm, w[i]);
    const float inc = wave_scan_max(lm);
    float Mp = fmaxf(M, dpp_ninf<0x138, 0xF>(inc));   // wave_shr:1 -> the exclusive prefix (lane 0: -inf)
    const float Mn = fmaxf(M, lane_f(inc, 63));
    // one expf per key, branch-free (lanes diverge on where the maxima fall):
    // a new maximum gives ms = expf(Mold - M) (0 before the first key), stored
    // negated (its vs = 1); any other key vs = expf(s - M)
    bool nm = false;
    uint32_t kb = 0;
#pragma unroll
    for (int i = 0; i < DX_B; i++) {
        const float s = w[i];
        const bool gt = s > Mp;
        const float e = expf(gt ? Mp - s : s - Mp);
        w[i] = gt ? -e : (s != -INFINITY ? e : 0.0f);
        Mp = fmaxf(Mp, s);
        nm = nm || gt;
        kb |= (uint32_t)gt << i;
    }
    if (kbits) *kbits = kb;
    // the lane's sequential S = S * ms + vs, (ms, vs) recovered from the signed
    // weight (a second pass: the first keeps only w[] live)
    float Sl = 0.0f, wl = 0.0f;
#pragma unroll
    for (int i = 0; i < DX_B; i++) {
        const float x = w[i];
        Sl = __builtin_signbit(x) ? fadd_rn(fmul_rn(Sl, -x), 1.0f) : fadd_rn(fmul_rn(Sl, 1.0f), x);
        if (lane * DX_B + i == n - 1) wl = x;
    }
    const float S = wave_sum(Mp == -INFINITY ? 0.0f : Sl * expf(Mp - Mn));
    flags = __ballot(nm || (lane + 1) * DX_B > n);   // (a batch with keys past n: the slow path, zero weights)
    wlast = lane_f(wl, (n - 1) / DX_B);
    M = Mn;
    return S;
}

}  // namespace qasr
