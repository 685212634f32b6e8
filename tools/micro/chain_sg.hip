// Micro-benchmark: cycles per key of the decode chain's inner block (8 keys)
// by where the key weights come from, V in registers (no memory traffic):
//   0: weights in fixed VGPRs              (mix + cvt)
//   1: weights in fixed SGPRs              (mix + cvt, SGPR operand)
//   2: SGPR weights by v_readlane in-block (mix + readlane + cvt: fx_pipe.h)
//   3: as 2 + the sequential fp32 S add    (v_add_f32 S, S, w)
//   4: VGPR weights by ds_read_b128 broadcast one group ahead (LDS)
//   5: as 4 + the sequential S add
//   6: single-rounding chain, VGPR weights (v_fma_mixlo_f16: one op a key)
//   7: as 2, readlanes batched at the group's start
//   8/9: LDS broadcast 1 / 2 groups ahead without the memory clobber
//   17/18: mixlo with LDS weights one / two groups ahead; 19: mixlo, two dimensions a lane;
//   20/21: two rows x two dimensions (the prefill chain) by mix/cvt_pk and by mixlo
//   13/14: two dimensions a lane (packed accumulator, v_cvt_pk_f16_f32), LDS / SGPR weights
//   10/12: weights by s_load_dwordx8 (glc / K$) one group ahead; 11: x16 glc, 16-key double buffer
// One wave per SIMD (8 workgroups of 4 waves), clock64 around 1024 groups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../qwen3-asr.cpp_amd/csrc/dev_common.h"


#define G 1024

#define MIXV(VI, W, SEL) "v_fma_mix_f32 %[t], " VI ", " W ", %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
#define CVT "v_cvt_f16_f32 %[a], %[t]\n\t"

template <int MODE>
__global__ __launch_bounds__(256) void k(const u32x4 *vin, const float *win, long long *cyc, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) float ws[4][64 + 16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    u32x4 v = vin[lane];
    float wl = win[lane];   // lane = key: the buffer's weights
    ws[wid][lane] = wl;
    if (lane < 16) ws[wid][64 + lane] = wl;
    __syncthreads();
    floatx4 wa = *(const floatx4 *)&ws[wid][0], wb = *(const floatx4 *)&ws[wid][4];
    int s0 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 0), s1 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 1),
        s2 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 2), s3 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 3),
        s4 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 4), s5 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 5),
        s6 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 6), s7 = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), 7);
    floatx4 wc = *(const floatx4 *)&ws[wid][8], wd = *(const floatx4 *)&ws[wid][12];
    typedef int int16v __attribute__((ext_vector_type(16)));
    int16v cur;
    for (int i = 0; i < 16; i++) cur[i] = __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl), i);
    f16 acc = 0;
    float S = 0.0f;
    const long long t0 = clock64();
    for (int g = 0; g < G; g++) {
        float t;
        if constexpr (MODE == 0) {
            asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT MIXV("%[v1]", "%[w2]", "0") CVT
                         MIXV("%[v1]", "%[w3]", "1") CVT MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                         MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                         : [t] "=&v"(t), [a] "+v"(acc)
                         : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                           [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3]));
        } else if constexpr (MODE == 1) {
            asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT MIXV("%[v1]", "%[w2]", "0") CVT
                         MIXV("%[v1]", "%[w3]", "1") CVT MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                         MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                         : [t] "=&v"(t), [a] "+v"(acc)
                         : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1), [w2] "s"(s2),
                           [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7));
        } else if constexpr (MODE == 2 || MODE == 3 || MODE == 7) {
            int n0, n1, n2, n3, n4, n5, n6, n7;
#define RL(N, L) "v_readlane_b32 %[" N "], %[wn], " #L "\n\t"
#define SADD(W) "v_add_f32 %[S], " W ", %[S]\n\t"
            if constexpr (MODE == 2)
                asm volatile(MIXV("%[v0]", "%[w0]", "0") RL("n0", 8) CVT MIXV("%[v0]", "%[w1]", "1") RL("n1", 9) CVT
                             MIXV("%[v1]", "%[w2]", "0") RL("n2", 10) CVT MIXV("%[v1]", "%[w3]", "1") RL("n3", 11) CVT
                             MIXV("%[v2]", "%[w4]", "0") RL("n4", 12) CVT MIXV("%[v2]", "%[w5]", "1") RL("n5", 13) CVT
                             MIXV("%[v3]", "%[w6]", "0") RL("n6", 14) CVT MIXV("%[v3]", "%[w7]", "1") RL("n7", 15) CVT
                             : [t] "=&v"(t), [a] "+v"(acc), [n0] "=&s"(n0), [n1] "=&s"(n1), [n2] "=&s"(n2), [n3] "=&s"(n3),
                               [n4] "=&s"(n4), [n5] "=&s"(n5), [n6] "=&s"(n6), [n7] "=&s"(n7)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1),
                               [w2] "s"(s2), [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7), [wn] "v"(wl));
            else if constexpr (MODE == 3)
                asm volatile(MIXV("%[v0]", "%[w0]", "0") RL("n0", 8) CVT SADD("%[w0]") MIXV("%[v0]", "%[w1]", "1") RL("n1", 9) CVT SADD("%[w1]")
                             MIXV("%[v1]", "%[w2]", "0") RL("n2", 10) CVT SADD("%[w2]") MIXV("%[v1]", "%[w3]", "1") RL("n3", 11) CVT SADD("%[w3]")
                             MIXV("%[v2]", "%[w4]", "0") RL("n4", 12) CVT SADD("%[w4]") MIXV("%[v2]", "%[w5]", "1") RL("n5", 13) CVT SADD("%[w5]")
                             MIXV("%[v3]", "%[w6]", "0") RL("n6", 14) CVT SADD("%[w6]") MIXV("%[v3]", "%[w7]", "1") RL("n7", 15) CVT SADD("%[w7]")
                             : [t] "=&v"(t), [a] "+v"(acc), [S] "+v"(S), [n0] "=&s"(n0), [n1] "=&s"(n1), [n2] "=&s"(n2), [n3] "=&s"(n3),
                               [n4] "=&s"(n4), [n5] "=&s"(n5), [n6] "=&s"(n6), [n7] "=&s"(n7)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1),
                               [w2] "s"(s2), [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7), [wn] "v"(wl));
            else
                asm volatile(RL("n0", 8) RL("n1", 9) RL("n2", 10) RL("n3", 11) RL("n4", 12) RL("n5", 13) RL("n6", 14) RL("n7", 15)
                             MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT
                             MIXV("%[v1]", "%[w2]", "0") CVT MIXV("%[v1]", "%[w3]", "1") CVT
                             MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                             MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                             : [t] "=&v"(t), [a] "+v"(acc), [n0] "=&s"(n0), [n1] "=&s"(n1), [n2] "=&s"(n2), [n3] "=&s"(n3),
                               [n4] "=&s"(n4), [n5] "=&s"(n5), [n6] "=&s"(n6), [n7] "=&s"(n7)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1),
                               [w2] "s"(s2), [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7), [wn] "v"(wl));
            s0 = n0; s1 = n1; s2 = n2; s3 = n3; s4 = n4; s5 = n5; s6 = n6; s7 = n7;
        } else if constexpr (MODE == 4 || MODE == 5) {
            const int o = (g & 7) * 8;
            const floatx4 na = *(const floatx4 *)&ws[wid][o + 8], nb = *(const floatx4 *)&ws[wid][o + 12];
            if constexpr (MODE == 4)
                asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT MIXV("%[v1]", "%[w2]", "0") CVT
                             MIXV("%[v1]", "%[w3]", "1") CVT MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                             MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                             : [t] "=&v"(t), [a] "+v"(acc)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                               [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3])
                             : "memory");
            else
                asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT SADD("%[w0]") MIXV("%[v0]", "%[w1]", "1") CVT SADD("%[w1]")
                             MIXV("%[v1]", "%[w2]", "0") CVT SADD("%[w2]") MIXV("%[v1]", "%[w3]", "1") CVT SADD("%[w3]")
                             MIXV("%[v2]", "%[w4]", "0") CVT SADD("%[w4]") MIXV("%[v2]", "%[w5]", "1") CVT SADD("%[w5]")
                             MIXV("%[v3]", "%[w6]", "0") CVT SADD("%[w6]") MIXV("%[v3]", "%[w7]", "1") CVT SADD("%[w7]")
                             : [t] "=&v"(t), [a] "+v"(acc), [S] "+v"(S)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                               [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3])
                             : "memory");
            wa = na;
            wb = nb;
        } else if constexpr (MODE == 8 || MODE == 9) {
            // LDS broadcast, no "memory" clobber; MODE 9: two groups ahead
            constexpr int AH = MODE == 8 ? 1 : 2;
            const int o = ((g + AH) & 7) * 8;
            const floatx4 na = *(const floatx4 *)&ws[wid][o], nb = *(const floatx4 *)&ws[wid][o + 4];
            asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT MIXV("%[v1]", "%[w2]", "0") CVT
                         MIXV("%[v1]", "%[w3]", "1") CVT MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                         MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                         : [t] "=&v"(t), [a] "+v"(acc)
                         : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                           [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3]));
            if constexpr (MODE == 8) {
                wa = na;
                wb = nb;
            } else {
                wa = wc;
                wb = wd;
                wc = na;
                wd = nb;
            }
        } else if constexpr (MODE >= 10 && MODE <= 12) {
            // SMEM: the weights from global memory by s_load into SGPRs; MODE 10: one
            // group (x8) ahead, glc; 11: 16 keys (x16) double-buffered, glc; 12: as 10 without glc
            if constexpr (MODE == 10 || MODE == 12) {
                int n0, n1, n2, n3, n4, n5, n6, n7;
                const float *src = win + ((g + 1) & 7) * 8;
                asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT MIXV("%[v1]", "%[w2]", "0") CVT
                             MIXV("%[v1]", "%[w3]", "1") CVT MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                             MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                             : [t] "=&v"(t), [a] "+v"(acc)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1),
                               [w2] "s"(s2), [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7));
                typedef int int8v __attribute__((ext_vector_type(8)));
                int8v r;
                if constexpr (MODE == 10) asm volatile("s_load_dwordx8 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(src));
                else asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(src));
                n0 = r[0]; n1 = r[1]; n2 = r[2]; n3 = r[3]; n4 = r[4]; n5 = r[5]; n6 = r[6]; n7 = r[7];
                s0 = n0; s1 = n1; s2 = n2; s3 = n3; s4 = n4; s5 = n5; s6 = n6; s7 = n7;
            } else {
                // 16 keys per batch: issue the next batch's x16 load, run 16 keys, then wait
                typedef int int16v __attribute__((ext_vector_type(16)));
                int16v nx;
                const float *src = win + ((g + 2) & 7) * 8;
                asm volatile("s_load_dwordx16 %0, %1, 0x0 glc" : "=s"(nx) : "s"(src));
                for (int h = 0; h < 2; h++) {
                    asm volatile(MIXV("%[v0]", "%[w0]", "0") CVT MIXV("%[v0]", "%[w1]", "1") CVT MIXV("%[v1]", "%[w2]", "0") CVT
                                 MIXV("%[v1]", "%[w3]", "1") CVT MIXV("%[v2]", "%[w4]", "0") CVT MIXV("%[v2]", "%[w5]", "1") CVT
                                 MIXV("%[v3]", "%[w6]", "0") CVT MIXV("%[v3]", "%[w7]", "1") CVT
                                 : [t] "=&v"(t), [a] "+v"(acc)
                                 : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(cur[8 * h + 0]),
                                   [w1] "s"(cur[8 * h + 1]), [w2] "s"(cur[8 * h + 2]), [w3] "s"(cur[8 * h + 3]),
                                   [w4] "s"(cur[8 * h + 4]), [w5] "s"(cur[8 * h + 5]), [w6] "s"(cur[8 * h + 6]),
                                   [w7] "s"(cur[8 * h + 7]));
                }
                asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(nx));
                cur = nx;
                g++;
            }
        } else if constexpr (MODE == 13 || MODE == 14) {
            // two dimensions a lane (d, d + 64) in one packed accumulator: per key
            // two mixes (lo / hi halves of acc as the fp16 addend) and one v_cvt_pk_f16_f32;
            // 13: VGPR weights by LDS broadcast one group ahead; 14: fixed SGPR weights
#define MIX2(VA, VB, W, SEL)                                                                     \
    "v_fma_mix_f32 %[t], " VA ", " W ", %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"        \
    "v_fma_mix_f32 %[u], " VB ", " W ", %[a] op_sel:[" SEL ",0,1] op_sel_hi:[1,0,1]\n\t"        \
    "v_cvt_pk_f16_f32 %[a], %[t], %[u]\n\t"
            float u;
            uint32_t a2 = __builtin_bit_cast(uint16_t, acc) * 0x10001u;
            if constexpr (MODE == 13) {
                const int o = ((g + 1) & 7) * 8;
                const floatx4 na = *(const floatx4 *)&ws[wid][o], nb = *(const floatx4 *)&ws[wid][o + 4];
                asm volatile(MIX2("%[v0]", "%[y0]", "%[w0]", "0") MIX2("%[v0]", "%[y0]", "%[w1]", "1")
                             MIX2("%[v1]", "%[y1]", "%[w2]", "0") MIX2("%[v1]", "%[y1]", "%[w3]", "1")
                             MIX2("%[v2]", "%[y2]", "%[w4]", "0") MIX2("%[v2]", "%[y2]", "%[w5]", "1")
                             MIX2("%[v3]", "%[y3]", "%[w6]", "0") MIX2("%[v3]", "%[y3]", "%[w7]", "1")
                             : [t] "=&v"(t), [u] "=&v"(u), [a] "+v"(a2)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [y0] "v"(v[1]), [y1] "v"(v[2]),
                               [y2] "v"(v[3]), [y3] "v"(v[0]), [w0] "v"(wa[0]), [w1] "v"(wa[1]), [w2] "v"(wa[2]), [w3] "v"(wa[3]),
                               [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3]));
                wa = na;
                wb = nb;
            } else {
                asm volatile(MIX2("%[v0]", "%[y0]", "%[w0]", "0") MIX2("%[v0]", "%[y0]", "%[w1]", "1")
                             MIX2("%[v1]", "%[y1]", "%[w2]", "0") MIX2("%[v1]", "%[y1]", "%[w3]", "1")
                             MIX2("%[v2]", "%[y2]", "%[w4]", "0") MIX2("%[v2]", "%[y2]", "%[w5]", "1")
                             MIX2("%[v3]", "%[y3]", "%[w6]", "0") MIX2("%[v3]", "%[y3]", "%[w7]", "1")
                             : [t] "=&v"(t), [u] "=&v"(u), [a] "+v"(a2)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [y0] "v"(v[1]), [y1] "v"(v[2]),
                               [y2] "v"(v[3]), [y3] "v"(v[0]), [w0] "s"(s0), [w1] "s"(s1), [w2] "s"(s2), [w3] "s"(s3),
                               [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7));
            }
            acc = __builtin_bit_cast(f16, (uint16_t)(a2 ^ (a2 >> 16)));
        } else if constexpr (MODE == 17 || MODE == 18) {
            // single rounding with the weights by LDS broadcast: 17 one group ahead
            // (as 4, memory clobber), 18 two groups ahead (as 9)
            constexpr int AH = MODE == 17 ? 1 : 2;
            const int o = ((g + AH) & 7) * 8;
            const floatx4 na = *(const floatx4 *)&ws[wid][o], nb = *(const floatx4 *)&ws[wid][o + 4];
#define MIXLO2(VI, W, SEL) "v_fma_mixlo_f16 %[a], " VI ", " W ", %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
            if constexpr (MODE == 17)
                asm volatile(MIXLO2("%[v0]", "%[w0]", "0") MIXLO2("%[v0]", "%[w1]", "1") MIXLO2("%[v1]", "%[w2]", "0")
                             MIXLO2("%[v1]", "%[w3]", "1") MIXLO2("%[v2]", "%[w4]", "0") MIXLO2("%[v2]", "%[w5]", "1")
                             MIXLO2("%[v3]", "%[w6]", "0") MIXLO2("%[v3]", "%[w7]", "1")
                             : [a] "+v"(acc)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                               [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3])
                             : "memory");
            else
                asm volatile(MIXLO2("%[v0]", "%[w0]", "0") MIXLO2("%[v0]", "%[w1]", "1") MIXLO2("%[v1]", "%[w2]", "0")
                             MIXLO2("%[v1]", "%[w3]", "1") MIXLO2("%[v2]", "%[w4]", "0") MIXLO2("%[v2]", "%[w5]", "1")
                             MIXLO2("%[v3]", "%[w6]", "0") MIXLO2("%[v3]", "%[w7]", "1")
                             : [a] "+v"(acc)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                               [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3]));
            if constexpr (AH == 1) {
                wa = na;
                wb = nb;
            } else {
                wa = wc;
                wb = wd;
                wc = na;
                wd = nb;
            }
            (void)t;
        } else if constexpr (MODE == 19 || MODE == 20 || MODE == 21) {
            // several independent chains a lane, per key: 19 two dimensions, one
            // mixlo each (separate registers); 20 two rows x two dimensions as the
            // prefill chain (mix, mix, cvt_pk per row); 21 the same four chains by mixlo
            uint32_t c0 = __builtin_bit_cast(uint16_t, acc), c1 = c0 ^ 1u, c2 = c0 ^ 2u, c3 = c0 ^ 3u;
#define ML(A, VI, W, SEL) "v_fma_mixlo_f16 " A ", " VI ", " W ", " A " op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
#define K19(VI, VJ, W, SEL) ML("%[c0]", VI, W, SEL) ML("%[c1]", VJ, W, SEL)
#define K21(VI, VJ, W, SEL) ML("%[c0]", VI, W, SEL) ML("%[c1]", VJ, W, SEL) ML("%[c2]", VI, W, SEL) ML("%[c3]", VJ, W, SEL)
#define K20(VA, VB, W, SEL)                                                                     \
    "v_fma_mix_f32 %[t], " VA ", " W ", %[c0] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"        \
    "v_fma_mix_f32 %[u], " VB ", " W ", %[c0] op_sel:[" SEL ",0,1] op_sel_hi:[1,0,1]\n\t"        \
    "v_cvt_pk_f16_f32 %[c0], %[t], %[u]\n\t"                                                     \
    "v_fma_mix_f32 %[t], " VA ", " W ", %[c1] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"        \
    "v_fma_mix_f32 %[u], " VB ", " W ", %[c1] op_sel:[" SEL ",0,1] op_sel_hi:[1,0,1]\n\t"        \
    "v_cvt_pk_f16_f32 %[c1], %[t], %[u]\n\t"
            float u;
            if constexpr (MODE == 19)
                asm volatile(K19("%[v0]", "%[v1]", "%[w0]", "0") K19("%[v0]", "%[v1]", "%[w1]", "1") K19("%[v1]", "%[v2]", "%[w2]", "0")
                             K19("%[v1]", "%[v2]", "%[w3]", "1") K19("%[v2]", "%[v3]", "%[w4]", "0") K19("%[v2]", "%[v3]", "%[w5]", "1")
                             K19("%[v3]", "%[v0]", "%[w6]", "0") K19("%[v3]", "%[v0]", "%[w7]", "1")
                             : [c0] "+v"(c0), [c1] "+v"(c1)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1), [w2] "s"(s2),
                               [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7));
            else if constexpr (MODE == 20)
                asm volatile(K20("%[v0]", "%[v1]", "%[w0]", "0") K20("%[v0]", "%[v1]", "%[w1]", "1") K20("%[v1]", "%[v2]", "%[w2]", "0")
                             K20("%[v1]", "%[v2]", "%[w3]", "1") K20("%[v2]", "%[v3]", "%[w4]", "0") K20("%[v2]", "%[v3]", "%[w5]", "1")
                             K20("%[v3]", "%[v0]", "%[w6]", "0") K20("%[v3]", "%[v0]", "%[w7]", "1")
                             : [c0] "+v"(c0), [c1] "+v"(c1), [t] "=&v"(t), [u] "=&v"(u)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1), [w2] "s"(s2),
                               [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7));
            else
                asm volatile(K21("%[v0]", "%[v1]", "%[w0]", "0") K21("%[v0]", "%[v1]", "%[w1]", "1") K21("%[v1]", "%[v2]", "%[w2]", "0")
                             K21("%[v1]", "%[v2]", "%[w3]", "1") K21("%[v2]", "%[v3]", "%[w4]", "0") K21("%[v2]", "%[v3]", "%[w5]", "1")
                             K21("%[v3]", "%[v0]", "%[w6]", "0") K21("%[v3]", "%[v0]", "%[w7]", "1")
                             : [c0] "+v"(c0), [c1] "+v"(c1), [c2] "+v"(c2), [c3] "+v"(c3)
                             : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "s"(s0), [w1] "s"(s1), [w2] "s"(s2),
                               [w3] "s"(s3), [w4] "s"(s4), [w5] "s"(s5), [w6] "s"(s6), [w7] "s"(s7));
            acc = __builtin_bit_cast(f16, (uint16_t)(c0 ^ c1 ^ c2 ^ c3));
        } else if constexpr (MODE == 6) {
#define MIXLO(VI, W, SEL) "v_fma_mixlo_f16 %[a], " VI ", " W ", %[a] op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
            asm volatile(MIXLO("%[v0]", "%[w0]", "0") MIXLO("%[v0]", "%[w1]", "1") MIXLO("%[v1]", "%[w2]", "0")
                         MIXLO("%[v1]", "%[w3]", "1") MIXLO("%[v2]", "%[w4]", "0") MIXLO("%[v2]", "%[w5]", "1")
                         MIXLO("%[v3]", "%[w6]", "0") MIXLO("%[v3]", "%[w7]", "1")
                         : [a] "+v"(acc)
                         : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [w0] "v"(wa[0]), [w1] "v"(wa[1]),
                           [w2] "v"(wa[2]), [w3] "v"(wa[3]), [w4] "v"(wb[0]), [w5] "v"(wb[1]), [w6] "v"(wb[2]), [w7] "v"(wb[3]));
            (void)t;
        }
    }
    const long long t1 = clock64();
    if (lane == 0) cyc[blockIdx.x * 4 + wid] = t1 - t0;
    out[(blockIdx.x * 4 + wid) * 64 + lane] = __builtin_bit_cast(uint16_t, acc) + __builtin_bit_cast(uint32_t, S);
}

int main() {
    u32x4 *v;
    float *w;
    long long *c;
    uint32_t *o;
    (void)hipMalloc(&v, 64 * 16);
    (void)hipMalloc(&w, 64 * 4);
    (void)hipMalloc(&c, 32 * 8);
    (void)hipMalloc(&o, 32 * 64 * 4);
    u32x4 hv[64];
    float hw[64];
    for (int i = 0; i < 64; i++) {
        hv[i] = u32x4{0x3c003c00u + i, 0x38003800u + i, 0x34003c00u + i, 0x3c003800u + i};
        hw[i] = 0.001f * (i + 1);
    }
    (void)hipMemcpy(v, hv, sizeof hv, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, hw, sizeof hw, hipMemcpyHostToDevice);
    const char *names[] = {"VGPR weights", "SGPR weights (fixed)", "SGPR by readlane in block", "readlane + S add",
                           "LDS broadcast one group ahead", "LDS + S add", "single rounding (mixlo), VGPR", "readlanes batched first",
                           "LDS 1 ahead, no clobber", "LDS 2 ahead, no clobber", "SMEM x8 glc, wait each group", "SMEM x16 glc, 16-key double buffer",
                           "SMEM x8 no glc (K$ hits)", "2 dims a lane, LDS weights", "2 dims a lane, SGPR weights",
                           "(removed: fx_pipe.h)", "(removed: fx_pipe.h)",
                           "mixlo, LDS 1 ahead", "mixlo, LDS 2 ahead", "mixlo, 2 dims (2 instr/key)",
                           "2 rows x 2 dims mix/cvt_pk (6/key)", "2 rows x 2 dims mixlo (4/key)"};
    for (int mode = 0; mode < 22; mode++) {
        double best = 1e30;
        for (int rep = 0; rep < 4; rep++) {
            switch (mode) {
            case 0: hipLaunchKernelGGL(k<0>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 1: hipLaunchKernelGGL(k<1>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 2: hipLaunchKernelGGL(k<2>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 3: hipLaunchKernelGGL(k<3>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 4: hipLaunchKernelGGL(k<4>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 5: hipLaunchKernelGGL(k<5>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 6: hipLaunchKernelGGL(k<6>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 7: hipLaunchKernelGGL(k<7>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 8: hipLaunchKernelGGL(k<8>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 9: hipLaunchKernelGGL(k<9>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 10: hipLaunchKernelGGL(k<10>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 11: hipLaunchKernelGGL(k<11>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 12: hipLaunchKernelGGL(k<12>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 13: hipLaunchKernelGGL(k<13>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 14: hipLaunchKernelGGL(k<14>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 15: case 16: continue;   // (fx_pipe.h's buffer, removed in round 5)
            case 17: hipLaunchKernelGGL(k<17>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 18: hipLaunchKernelGGL(k<18>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 19: hipLaunchKernelGGL(k<19>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 20: hipLaunchKernelGGL(k<20>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            case 21: hipLaunchKernelGGL(k<21>, dim3(8), dim3(256), 0, 0, v, w, c, o); break;
            }
            (void)hipDeviceSynchronize();
            long long hc[32];
            (void)hipMemcpy(hc, c, sizeof hc, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < 32; i++) s += hc[i];
            s /= 32;
            best = s < best ? s : best;
        }
        printf("mode %d  %-32s %6.2f cycles/key\n", mode, names[mode], best / (8.0 * G));
    }
    return 0;
}
