// dev_common.h -- shared device helpers for the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64

__device__ __forceinline__ float h2f(f16 h) { return (float)h; }
// The fp32 value as rounded, opaque to the optimiser.  Without it LLVM folds
// fptrunc(fmul/fadd) into v_fma_mixlo_f16, which rounds the product straight
// to fp16 -- one rounding where ggml (and the reference) round to fp32 first
// and then to fp16: the two differ on rare ties, and a kernel that got the
// fold disagreed with one that did not (measured: tools/diag_fused2.py, one
// fp16 ulp on 386 of 3072 SwiGLU outputs at decoder layer 18).
__device__ __forceinline__ float rn32(float f) {
    asm("" : "+v"(f));
    return f;
}
// fp32 -> fp16 round-to-nearest-even (v_cvt_f16_f32 under the default mode),
// identical to ggml's GGML_CPU_FP32_TO_FP16 / F16C _cvtss_sh(x, 0).
__device__ __forceinline__ f16 f2h(float f) { return (f16)rn32(f); }
__device__ __forceinline__ float u16_to_f(uint16_t u) { return (float)__builtin_bit_cast(f16, u); }
__device__ __forceinline__ uint16_t f_to_u16(float f) { return __builtin_bit_cast(uint16_t, (f16)rn32(f)); }

// 100 MHz constant clock shared by all CUs (dev trace timestamps)
__device__ __forceinline__ unsigned long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void trace_mark(unsigned long long *tr, int slot) {
    if (tr && threadIdx.x == 0) tr[(long)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + slot] = rt_now();
}

// kernel-duration probe (qasr_set_probe): lane 0 of each workgroup folds its
// start / end time (the 100 MHz clock) into shard blockIdx % 32 of a
// per-launch record: min-starts at st[32 * shard], max-ends at
// st[STAMP_ENDS + 32 * shard] -- every shard on a 256-B line of its own (one
// line taking every block's atomic serialised them at the memory side: +6 us
// on a 1024-block launch); no-return atomics, 32 per line; null (one untaken
// branch) unless this launch is probed
#define STAMP_ENDS (32 * 32)
__device__ __forceinline__ void stamp_start(unsigned long long *st) {
    if (st && threadIdx.x == 0) atomicMin(st + 32 * (blockIdx.x & 31), rt_now());
}
__device__ __forceinline__ void stamp_end(unsigned long long *st) {
    if (st && threadIdx.x == 0) atomicMax(st + STAMP_ENDS + 32 * (blockIdx.x & 31), rt_now());
}

// DPP lane moves (VALU, no LDS round trip): quad_perm xor1 / xor2, row half
// mirror (lane i <-> 7-i in 8), row mirror (lane i <-> 15-i in 16)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// every lane of each 16-lane row receives the row's sum / max
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    return v;
}
__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    v = fmaxf(v, dpp_f<0x140>(v));
    return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// wave64 reductions: rows by DPP, then the four row results by readlane
// (uniform result in every lane)
__device__ __forceinline__ float wave_sum(float v) {
    v = row16_sum(v);
    return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    v = row16_max(v);
    return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// total order on finite doubles as unsigned 64-bit keys (for atomicMax)
__device__ __forceinline__ unsigned long long dkey(double d) {
    unsigned long long u = __double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(unsigned long long k) {
    unsigned long long u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double(u);
}
// argmax key: larger value wins, ties -> lower index (src/qwen3_asr.cpp:309-313 strict '>')
__device__ __forceinline__ unsigned long long argmax_key(float v, int idx) {
    uint32_t u = __float_as_uint(v);
    u = (u >> 31) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned long long)(0xffffffffu - (uint32_t)idx);
}
__device__ __forceinline__ int argmax_key_idx(unsigned long long k) { return (int)(0xffffffffu - (uint32_t)(k & 0xffffffffu)); }

// non-contracted fp32 ops (ggml computes these as separate ops, each rounded)
__device__ __forceinline__ float fmul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub_rn(float a, float b) { return __fsub_rn(a, b); }

// ggml tanh-GELU through the fp16 table (GGML_GELU_FP16)
__device__ __forceinline__ float gelu_lut(float x, const uint16_t *__restrict__ lut) {
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return u16_to_f(lut[f_to_u16(x)]);
}
// the same, as the fp16 bits of the result (what a following fp16 store writes)
__device__ __forceinline__ uint32_t gelu_lut_bits(float x, const uint16_t *__restrict__ lut) {
    if (x <= -10.0f) return 0u;
    if (x >= 10.0f) return f_to_u16(x);
    return lut[f_to_u16(x)];
}

// ggml quantize_row_q8_0 (x86 path) for one value of a 32-block whose |max| is
// amax: d = fp16(amax / 127), q = round-half-even(v * 127 / amax)
// (quantize_q8_kernel, elementwise.hip, is the reference restatement)
__device__ __forceinline__ float q8_scale(float amax) { return u16_to_f(f_to_u16(amax / 127.f)); }
__device__ __forceinline__ int8_t q8_quant(float v, float amax) {
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    return (int8_t)__builtin_rintf(fmul_rn(v, id));
}

typedef int intx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

// acc[r] += (d_w * d_x[r]) * sumi[r]: the scale products and the fma in
// packed fp32 (v_pk_mul_f32 / v_pk_fma_f32, two rows per instruction; each
// lane's arithmetic and rounding identical to the scalar fmul + fma)
__device__ __forceinline__ void q8_scale_acc(floatx4 &acc, float dw, floatx4 dx, intx4 ci) {
    const floatx2 w2 = {dw, dw};
    const floatx2 s01 = w2 * floatx2{dx[0], dx[1]}, s23 = w2 * floatx2{dx[2], dx[3]};
    const floatx2 c01 = {(float)ci[0], (float)ci[1]}, c23 = {(float)ci[2], (float)ci[3]};
    const floatx2 a01 = __builtin_elementwise_fma(s01, c01, floatx2{acc[0], acc[1]});
    const floatx2 a23 = __builtin_elementwise_fma(s23, c23, floatx2{acc[2], acc[3]});
    acc = floatx4{a01[0], a01[1], a23[0], a23[1]};
}

// ggml_rms_norm (+ mul by w) of one D-wide fp32 row by one wave: lane owns
// columns 4 lane + 256 i (v[i]); sum of fp32 squares in double, scale =
// 1/sqrtf(mean + eps).  Output: fp16 y, fp32 y32, or Q8_0 (yq int8 + yd fp32
// block scales, a 32-block = 8 lanes) -- row `row` of a D-wide output.
// Shared by rmsnorm_kernel and the skinny GEMM's fused post-norm, so both give
// the same bits.
template <int D>
__device__ __forceinline__ void rms_row(const float4 *v, const float *__restrict__ w, float eps, long row,
                                        uint16_t *__restrict__ y, float *__restrict__ y32, int8_t *__restrict__ yq,
                                        float *__restrict__ yd) {
    constexpr int PER = D / 256;
    const int lane = threadIdx.x & 63;
    float4 wv[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) wv[i] = *(const float4 *)(w + 4 * lane + 256 * i);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < PER; i++)
        s += ((double)fmul_rn(v[i].x, v[i].x) + (double)fmul_rn(v[i].y, v[i].y)) +
             ((double)fmul_rn(v[i].z, v[i].z) + (double)fmul_rn(v[i].w, v[i].w));
    s = wave_sum_d(s);
    const float mean = (float)(s / D);
    const float scale = 1.0f / sqrtf(mean + eps);
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const float4 t = make_float4(fmul_rn(fmul_rn(v[i].x, scale), wv[i].x), fmul_rn(fmul_rn(v[i].y, scale), wv[i].y),
                                     fmul_rn(fmul_rn(v[i].z, scale), wv[i].z), fmul_rn(fmul_rn(v[i].w, scale), wv[i].w));
        const long o = row * D + 4 * lane + 256 * i;
        if (yq) {
            float am = fmaxf(fmaxf(fabsf(t.x), fabsf(t.y)), fmaxf(fabsf(t.z), fabsf(t.w)));
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            am = fmaxf(am, __shfl_xor(am, 2, 64));
            am = fmaxf(am, __shfl_xor(am, 4, 64));
            const uint32_t u = (uint32_t)(uint8_t)q8_quant(t.x, am) | (uint32_t)(uint8_t)q8_quant(t.y, am) << 8 |
                               (uint32_t)(uint8_t)q8_quant(t.z, am) << 16 | (uint32_t)(uint8_t)q8_quant(t.w, am) << 24;
            *(uint32_t *)(yq + o) = u;
            if ((lane & 7) == 0) yd[row * (D / 32) + lane / 8 + 8 * i] = q8_scale(am);
        } else if (y32) {
            *(float4 *)(y32 + o) = t;
        } else {
            const uint32_t lo = f_to_u16(t.x) | ((uint32_t)f_to_u16(t.y) << 16), hi = f_to_u16(t.z) | ((uint32_t)f_to_u16(t.w) << 16);
            *(uint2 *)(y + o) = make_uint2(lo, hi);
        }
    }
}
