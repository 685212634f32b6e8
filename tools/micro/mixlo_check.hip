// Bit check of the two fp16 V-accumulator steps on gfx950 against the
// oracle's restatements (oracle/qasr_oracle.c):
//   r2: v_fma_mix_f32 + v_cvt_f16_f32        == qo_f16_mad_round2 (ggml F16C)
//   r1: v_fma_mixlo_f16 (one rounding)       == qo_f16_mad_round1 (QO_FA_V_ROUND1)
//   r1 scale: v_fma_mixlo_f16 acc * ms + 0   (reported only)
// over random triples (fp16 x and y over the whole finite range incl.
// subnormals, fp32 v in [0, 1], exp(-U(0,30)) and tiny) plus 256-key chains.
// Build: hipcc --offload-arch=gfx950 -O2 mixlo_check.hip -I../../oracle -L../../oracle -loracle -Wl,-rpath,$ORIGIN/../../oracle
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "qasr_oracle.h"

__global__ void steps(const uint16_t *x, const float *v, const uint16_t *y, uint16_t *o1, uint16_t *o2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t a1 = y[i], xv = x[i];
    const float vs = v[i];
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a1) : "v"(xv), "v"(vs));
    float t;
    uint32_t a2 = y[i];
    asm volatile("v_fma_mix_f32 %0, %2, %3, %1 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32 %1, %0" : "=&v"(t), "+v"(a2) : "v"(xv), "v"(vs));
    o1[i] = (uint16_t)a1;
    o2[i] = (uint16_t)a2;
}

// one chain of K keys per thread, both forms
__global__ void chains(const uint16_t *x, const float *v, uint16_t *o1, uint16_t *o2, int K, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t a1 = 0, a2 = 0;
    for (int k = 0; k < K; k++) {
        const uint32_t xv = x[(long)i * K + k];
        const float vs = v[(long)i * K + k];
        float t;
        asm volatile("v_fma_mixlo_f16 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a1) : "v"(xv), "v"(vs));
        asm volatile("v_fma_mix_f32 %0, %2, %3, %1 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32 %1, %0" : "=&v"(t), "+v"(a2) : "v"(xv), "v"(vs));
    }
    o1[i] = (uint16_t)a1;
    o2[i] = (uint16_t)a2;
}

static uint64_t rs = 88172645463325252ull;
static uint64_t xr() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}
static double ur() { return (xr() >> 11) * (1.0 / 9007199254740992.0); }
static uint16_t rh() {   // finite fp16, both signs
    uint16_t h;
    do h = (uint16_t)xr(); while ((h & 0x7c00u) == 0x7c00u);
    return h;
}
static float rv() {
    const int k = xr() % 3;
    return k == 0 ? (float)ur() : k == 1 ? expf(-30.0f * (float)ur()) : (float)(ur() * 1e-6);
}

int main() {
    const int N = 1 << 22;
    uint16_t *hx = (uint16_t *)malloc(N * 2), *hy = (uint16_t *)malloc(N * 2), *h1 = (uint16_t *)malloc(N * 2),
             *h2 = (uint16_t *)malloc(N * 2);
    float *hv = (float *)malloc(N * 4);
    for (int i = 0; i < N; i++) {
        hx[i] = rh();
        hy[i] = rh();
        hv[i] = rv();
    }
    // constructed double-rounding cases: y = 2^e, x = 1, v = 2^(e - 11) (1 + 2^-23) and negatives
    int m = 0;
    for (int e = -14; e <= 14 && m < 1024; e++)
        for (int s = 0; s < 2; s++) {
            hx[m] = 0x3c00 | (s << 15);
            hv[m] = ldexpf(1.0f + ldexpf(1.0f, -23), e - 11);
            hy[m] = (uint16_t)(((e + 15) << 10) | (s << 15));
            m++;
        }
    uint16_t *dx, *dy, *d1, *d2;
    float *dv;
    (void)hipMalloc(&dx, N * 2);
    (void)hipMalloc(&dy, N * 2);
    (void)hipMalloc(&d1, N * 2);
    (void)hipMalloc(&d2, N * 2);
    (void)hipMalloc(&dv, N * 4);
    (void)hipMemcpy(dx, hx, N * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dy, hy, N * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dv, hv, N * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(steps, dim3(N / 256), dim3(256), 0, 0, dx, dv, dy, d1, d2, N);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h1, d1, N * 2, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2, d2, N * 2, hipMemcpyDeviceToHost);
    long bad1 = 0, bad2 = 0, diff12 = 0;
    for (int i = 0; i < N; i++) {
        const uint16_t r1 = qo_f16_mad_round1(hx[i], hv[i], hy[i]), r2 = qo_f16_mad_round2(hx[i], hv[i], hy[i]);
        if (h1[i] != r1 && bad1++ < 8) printf("  r1 mismatch x=%04x v=%a y=%04x gpu=%04x oracle=%04x\n", hx[i], hv[i], hy[i], h1[i], r1);
        if (h2[i] != r2 && bad2++ < 8) printf("  r2 mismatch x=%04x v=%a y=%04x gpu=%04x oracle=%04x\n", hx[i], hv[i], hy[i], h2[i], r2);
        diff12 += r1 != r2;
    }
    printf("steps: %d triples, round1 mismatches %ld, round2 mismatches %ld, round1 != round2 in %ld\n", N, bad1, bad2, diff12);
    // chains: 4096 threads x 256 keys, v in the attention-weight range, x ~ fp16 values of |v| < 4
    const int T = 4096, K = 256;
    for (long i = 0; i < (long)T * K; i++) {
        hx[i] = (uint16_t)((xr() & 0x8000u) | (0x3000u + xr() % 0x1400u));
        hv[i] = expf(-8.0f * (float)ur());
    }
    (void)hipMemcpy(dx, hx, (long)T * K * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dv, hv, (long)T * K * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chains, dim3(T / 256), dim3(256), 0, 0, dx, dv, d1, d2, K, T);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h1, d1, T * 2, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2, d2, T * 2, hipMemcpyDeviceToHost);
    long cb1 = 0, cb2 = 0, cd = 0;
    for (int t = 0; t < T; t++) {
        uint16_t a1 = 0, a2 = 0;
        for (int k = 0; k < K; k++) {
            a1 = qo_f16_mad_round1(hx[(long)t * K + k], hv[(long)t * K + k], a1);
            a2 = qo_f16_mad_round2(hx[(long)t * K + k], hv[(long)t * K + k], a2);
        }
        cb1 += a1 != h1[t];
        cb2 += a2 != h2[t];
        cd += a1 != a2;
    }
    printf("chains: %d x %d keys, round1 mismatches %ld, round2 mismatches %ld, final round1 != round2 in %ld\n", T, K, cb1, cb2, cd);
    return (bad1 || bad2 || cb1 || cb2) ? 1 : 0;
}
