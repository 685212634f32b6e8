// Micro-benchmark: cycles per key of the fp16-accumulator chain variants
// (fa_exact.hip) on one wave, values in registers, shader clock (s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16;
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f16 cvt_asm(float f) {
    f16 h;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(h) : "v"(f));
    return h;
}
__device__ __forceinline__ half2v mad2(half2v acc, uint32_t v, float vs) {
    const half2v vv = __builtin_bit_cast(half2v, v);
    const float f0 = fmaf((float)vv.x, vs, (float)acc.x);
    const float f1 = fmaf((float)vv.y, vs, (float)acc.y);
    return __builtin_convertvector((floatx2){f0, f1}, half2v);
}

template <int MODE>
__global__ void k(const uint32_t *vin, const float *win, float *out, long long *cyc, int n) {
    uint32_t v[16];
    float w[16];
    for (int i = 0; i < 16; i++) { v[i] = vin[i * 64 + threadIdx.x]; w[i] = win[i]; }
    float a32 = 0.f;
    f16 a16 = 0;
    half2v a2[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
    float a2f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __syncthreads();
    const long long t0 = clock64();
    for (int j = 0; j < n; j += 16) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if constexpr (MODE == 0) a32 = fmaf(__uint_as_float(v[i]), w[i], a32);
            if constexpr (MODE == 1) a16 = cvt_asm(fmaf((float)__builtin_bit_cast(f16, (uint16_t)v[i]), w[i], (float)a16));
            if constexpr (MODE == 2) a2[0] = mad2(a2[0], v[i], w[i]);
            if constexpr (MODE == 3)
#pragma unroll
                for (int r = 0; r < 4; r++) a2[r] = mad2(a2[r], v[i], w[(i + r) & 15]);
            if constexpr (MODE == 4)   // 8 independent fp32 fma chains: the plain VALU rate
#pragma unroll
                for (int r = 0; r < 8; r++) a2f[r] = fmaf(__uint_as_float(v[i]), w[(i + r) & 15], a2f[r]);
        }
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 64 + threadIdx.x] = a32 + (float)a16 + (float)a2[0].x + (float)a2[1].y + (float)a2[2].x + (float)a2[3].y + a2f[0] + a2f[1] + a2f[2] +
                                       a2f[3] + a2f[4] + a2f[5] + a2f[6] + a2f[7];
}

int main() {
    const int n = 1 << 16;
    uint32_t *v; float *w, *o; long long *c;
    hipMalloc(&v, 64 * 16 * 4); hipMalloc(&w, 64); hipMalloc(&o, 8192 * 64 * 4); hipMalloc(&c, 8192 * 8);
    hipMemset(v, 0x11, 64 * 16 * 4); hipMemset(w, 0, 64);
    const char *names[] = {"fp32 fma chain", "mix + asm cvt (1 dim)", "2x mix + cvt_pk (2 dims)", "4 rows x (2x mix + cvt_pk)",
                           "8 independent fp32 fma"};
    for (int mode = 0; mode < 5; mode++) {
        for (int blocks : {1, 1024, 2048, 4096, 8192}) {
            for (int rep = 0; rep < 2; rep++) {
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
                if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
                if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
                hipDeviceSynchronize();
            }
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0, 0);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
            if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
            if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, v, w, o, c, n);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            long long h;
            hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
            const int inst = mode == 0 ? 1 : mode == 1 ? 2 : mode == 2 ? 3 : mode == 3 ? 12 : 8;
            printf("%-32s waves=%5d  %.2f cycles/key/wave  %.3f wave-VALU/cycle/SIMD (2.4 GHz)\n", names[mode], blocks, (double)h / n,
                   (double)blocks * n * inst / 1024.0 / (ms * 1e-3 * 2.4e9));
        }
    }
    return 0;
}
