// store_pat.hip -- the 8-phase GEMM epilogue's store pattern in isolation: one
// workgroup of 8 waves per 256 x 256 fp32 output tile of a [M][N] row-major
// array, no loads, no MFMA.  A: as g8_epilogue (wave (wr, wc) writes its four
// 64 x 32 quadrants, 8 lanes a 128-B row segment, 8 rows a store); B: the same
// with nontemporal stores; C: each wave writes whole 1-KB tile rows (64 lanes x
// 16 B, one row a store).  Effective write rate = M * N * 4 B / time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void store_kernel(float *out, int M, int N) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;
    const int ntn = N >> 8, wg = blockIdx.x;
    const int m0 = (wg / ntn) * 256, n0 = (wg % ntn) * 256;
    const floatx4 v = floatx4{(float)lane, (float)wid, (float)m0, (float)n0};
    if constexpr (MODE == 2) {
#pragma unroll 4
        for (int r = 0; r < 32; r++) {
            const int row = m0 + wid * 32 + r;
            if (row < M) *(floatx4 *)(out + (long)row * N + n0 + 4 * lane) = v;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = q >> 1, j = q & 1;
            const int c0 = n0 + j * 128 + wc * 32, r0 = m0 + i * 128 + wr * 64;
            const int col = c0 + 4 * (lane & 7);
#pragma unroll
            for (int it = 0; it < 8; it++) {
                const int row = r0 + (lane >> 3) + 8 * it;
                if (row >= M) continue;
                floatx4 *p = (floatx4 *)(out + (long)row * N + col);
                if constexpr (MODE == 1) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
        }
    }
}

int main() {
    struct Sh { const char *name; int M, N; } shapes[] = {{"prefill qkv b64", 25920, 4096}, {"prefill gu b64", 25920, 6144},
                                                         {"prefill o b64", 25920, 1024}, {"enc qkv b64", 24960, 2816}};
    float *out;
    CK(hipMalloc(&out, (size_t)25920 * 6144 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (const Sh &sh : shapes) {
        const int tiles = ((sh.M + 255) / 256) * (sh.N / 256);
        printf("%s M=%d N=%d (%d tiles)\n", sh.name, sh.M, sh.N, tiles);
        for (int mode = 0; mode < 3; mode++) {
            auto launch = [&] {
                if (mode == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(tiles), dim3(512), 0, 0, out, sh.M, sh.N);
                if (mode == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(tiles), dim3(512), 0, 0, out, sh.M, sh.N);
                if (mode == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(tiles), dim3(512), 0, 0, out, sh.M, sh.N);
            };
            launch();
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipEventRecord(a, 0));
                for (int r = 0; r < 10; r++) launch();
                CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
                float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
            }
            const double us = best * 100.0, gb = (double)sh.M * sh.N * 4 / 1e9;
            printf("  %-28s %7.1f us %6.2f TB/s\n", mode == 0 ? "A quadrant 128-B segments" : mode == 1 ? "B same, nontemporal" : "C 1-KB rows", us,
                   gb / us * 1e3);
        }
    }
    return 0;
}
