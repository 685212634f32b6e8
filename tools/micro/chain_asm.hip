// Micro-benchmark + bit check: the decode chain step (fx_chain.h) written as
// one inline-asm block per 8 keys against the compiler-scheduled form.
//   mode 0: compiler form (v_fma_mix_f32 + asm v_cvt_f16_f32, weights in SGPRs by readlane)
//   mode 1: asm block, weights in VGPRs, no wait state between mix and cvt
//   mode 2: asm block, weights in VGPRs, s_nop 0 between mix and cvt
//   mode 3: asm block, weights in SGPRs (uniform loads), no wait state
//   mode 4: asm block, weights in SGPRs, s_nop 0
//   mode 5: asm block, weights per lane in a VGPR array, v_readlane'd into SGPRs (the register-weights form)
//   mode 6: asm block, VGPR weights from LDS (two uniform ds_read_b128 per 8 keys, one group ahead: the fused
//           launch's chain role, fx_chain.h fx_step1_lds)
// (modes 1 / 2 rebuild their VGPR weight operands from SGPRs inside the loop: v_movs the real kernel does not have)
// One wave per workgroup; cycles per key by s_memtime; every lane's final
// accumulator compared bit for bit with mode 0's.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef _Float16 f16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f16 cvt_asm(float f) {
    f16 h;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(h) : "v"(f));
    return h;
}

#define MIX(VI, W, SEL) "v_fma_mix_f32 %0, " VI ", " W ", %1 op_sel:[" SEL ",0,0] op_sel_hi:[1,0,1]\n\t"
#define CHAIN8(CVT)                                                                                                          \
    asm volatile(MIX("%2", "%6", "0") CVT MIX("%2", "%7", "1") CVT MIX("%3", "%8", "0") CVT MIX("%3", "%9", "1") CVT          \
                 MIX("%4", "%10", "0") CVT MIX("%4", "%11", "1") CVT MIX("%5", "%12", "0") CVT MIX("%5", "%13", "1") CVT   \
                 : "=&v"(t), "+v"(acc)                                                                                       \
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(wa[0]), "v"(wa[1]), "v"(wa[2]), "v"(wa[3]), "v"(wb[0]),  \
                   "v"(wb[1]), "v"(wb[2]), "v"(wb[3])                                                                        \
                 : "memory")
#define CHAIN8S(CVT)                                                                                                         \
    asm volatile(MIX("%2", "%6", "0") CVT MIX("%2", "%7", "1") CVT MIX("%3", "%8", "0") CVT MIX("%3", "%9", "1") CVT          \
                 MIX("%4", "%10", "0") CVT MIX("%4", "%11", "1") CVT MIX("%5", "%12", "0") CVT MIX("%5", "%13", "1") CVT   \
                 : "=&v"(t), "+v"(acc)                                                                                       \
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "s"(w[0]), "s"(w[1]), "s"(w[2]), "s"(w[3]), "s"(w[4]),       \
                   "s"(w[5]), "s"(w[6]), "s"(w[7])                                                                           \
                 : "memory")
template <int NOP>
__device__ __forceinline__ void chain8s(f16 &acc, u32x4 v, const float *w) {
    float t;
    if constexpr (NOP) CHAIN8S("s_nop 0\n\tv_cvt_f16_f32 %1, %0\n\t");
    else CHAIN8S("v_cvt_f16_f32 %1, %0\n\t");
}
template <int NOP>
__device__ __forceinline__ void chain8(f16 &acc, u32x4 v, floatx4 wa, floatx4 wb) {
    float t;
    if constexpr (NOP) CHAIN8("s_nop 0\n\tv_cvt_f16_f32 %1, %0\n\t");
    else CHAIN8("v_cvt_f16_f32 %1, %0\n\t");
}

template <int MODE>
__global__ void k(const u32x4 *vin, const float *win, uint16_t *out, long long *cyc, int n) {
    const int lane = threadIdx.x;
    __shared__ __attribute__((aligned(16))) float wlds[64 + 8];
    wlds[lane] = win[lane];
    if (lane < 8) wlds[64 + lane] = win[lane];
    u32x4 v[8];
    for (int i = 0; i < 8; i++) v[i] = vin[i * 64 + lane];
    float w[64];
    for (int i = 0; i < 64; i++) w[i] = win[i];
    float wl[4];   // mode 5: per-lane weights (lane l holds win[l] in every element)
    for (int i = 0; i < 4; i++) wl[i] = win[lane];
    f16 acc = 0;
    __syncthreads();
    const long long t0 = clock64();
    if constexpr (MODE == 6) {
        floatx4 wa = *(const floatx4 *)&wlds[0], wb = *(const floatx4 *)&wlds[4];
        for (int j = 0; j < n; j += 64) {
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const floatx4 na = *(const floatx4 *)&wlds[8 * b + 8], nb = *(const floatx4 *)&wlds[8 * b + 12];
                chain8<0>(acc, v[b], wa, wb);
                wa = na;
                wb = nb;
            }
        }
    } else
    for (int j = 0; j < n; j += 64) {
#pragma unroll
        for (int b = 0; b < 8; b++) {
            if constexpr (MODE == 0) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const uint32_t d = v[b][i >> 1];
                    const uint16_t e = (i & 1) ? (d >> 16) : (d & 0xffff);
                    acc = cvt_asm(fmaf((float)__builtin_bit_cast(f16, e), w[8 * b + i], (float)acc));
                }
            } else if constexpr (MODE == 6) {
                // (one group ahead: the loads of group b + 1 before the block of group b)
                static_assert(MODE == 6, "");
            } else if constexpr (MODE == 3 || MODE == 4) {
                chain8s<MODE == 4>(acc, v[b], w + 8 * b);
            } else if constexpr (MODE == 5) {
                float ws[8];
#pragma unroll
                for (int i = 0; i < 8; i++)
                    ws[i] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wl[i & 3]), (8 * b + i) & 63));
                chain8s<0>(acc, v[b], ws);
            } else {
                const floatx4 wa = {w[8 * b], w[8 * b + 1], w[8 * b + 2], w[8 * b + 3]};
                const floatx4 wb = {w[8 * b + 4], w[8 * b + 5], w[8 * b + 6], w[8 * b + 7]};
                chain8<MODE == 2>(acc, v[b], wa, wb);
            }
        }
    }
    const long long t1 = clock64();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 64 + lane] = __builtin_bit_cast(uint16_t, acc);
}

int main() {
    const int n = 1 << 14, blocks = 256;
    u32x4 *v; float *w; uint16_t *o; long long *c;
    (void)hipMalloc(&v, 8 * 64 * 16); (void)hipMalloc(&w, 64 * 4); (void)hipMalloc(&o, blocks * 64 * 2 * 3); (void)hipMalloc(&c, blocks * 8);
    unsigned hv[8 * 64 * 4];
    float hw[64];
    srand(7);
    for (auto &x : hv) {   // fp16 pairs in [-2, 2)
        const uint16_t a = (uint16_t)(((rand() & 0x1) << 15) | (0x3800 + (rand() % 0x800))), b = (uint16_t)(((rand() & 0x1) << 15) | (0x3800 + (rand() % 0x800)));
        x = a | ((unsigned)b << 16);
    }
    for (auto &x : hw) x = (float)rand() / RAND_MAX;
    (void)hipMemcpy(v, hv, sizeof hv, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, hw, sizeof hw, hipMemcpyHostToDevice);
    const char *names[] = {"compiler (mix + asm cvt)", "asm, VGPR weights, no nop", "asm, VGPR weights, s_nop 0",
                           "asm, SGPR weights, no nop", "asm, SGPR weights, s_nop 0", "asm, readlane'd weights, no nop",
                           "asm, LDS -> VGPR weights, no nop"};
    uint16_t ref[blocks * 64];
    for (int mode = 0; mode < 7; mode++) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        if (mode == 5) hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        if (mode == 6) hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
        (void)hipDeviceSynchronize();
        long long hc[blocks];
        uint16_t ho[blocks * 64];
        (void)hipMemcpy(hc, c, sizeof hc, hipMemcpyDeviceToHost);
        (void)hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
        if (mode == 0) memcpy(ref, ho, sizeof ho);
        long long s = 0;
        for (int b = 0; b < blocks; b++) s += hc[b];
        const int same = mode == 5 || mode == 6 || !memcmp(ref, ho, sizeof ho);   // (modes 5, 6: other weight order, speed only)
        printf("mode %d %-28s %.2f cycles/key  bit-identical to mode 0: %s\n", mode, names[mode], (double)s / blocks / n,
               same ? "yes" : "NO");
    }
    return 0;
}
