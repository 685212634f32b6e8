// Micro-benchmark: the fused launch's chain loop outside the fused kernel,
// to separate the loop's own cost from its environment (32 chain waves, 4 per
// workgroup, n = 1370 keys, V^T double-buffered from global memory).
//   mode 0: fx_step1_lds as built (flags at run time)
//   mode 1: fast path only (no slow-path code in the loop)
//   mode 2: fast path only, V^T not reloaded (first two buffers reused)
//   mode 3: as 2, and the weights not reloaded from LDS (fx8_fast on fixed registers)
//   mode 4: as 0 (V^T reloaded), weights not reloaded from LDS
//   mode 5: as 0 with the slow path per 8-key group (fx_step1_lds_m): argv[3]
//           = the 64-bit new-maximum mask of every 64-key buffer
//   argv[2] = waves per workgroup (4 or 1); argv[3] = the batches' slow-path flags (default 0)
// Prints cycles per key (s_memtime), mean over the chain waves.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../qwen3-asr.cpp_amd/csrc/fx_chain.h"

using namespace qasr;

template <int MODE>
__global__ __launch_bounds__(256) void chain_k(const uint16_t *vt_all, const float *wsrc, int n, long long *cyc, uint16_t *out,
                                               unsigned long long flags) {
    __shared__ __attribute__((aligned(16))) float ws[4][DX_KC / DX_B * FX_ST];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int i = lane; i < DX_KC / DX_B * FX_ST; i += 64) ws[wid][i] = wsrc[i];
    const int gw = blockIdx.x * (blockDim.x / 64) + wid;
    const uint16_t *vt = vt_all + (long)gw * 1024 * (DX_KC / 8 + 64);
    const int loff = 8 * lane;
    __syncthreads();
    f16 acc = 0;
    const long long t0 = clock64();
    u32x4 va[DX_Q / 8], vb[DX_Q / 8];
    fx_loadQ(va, vt, loff, 0);
    if constexpr (false) {
    } else {
        floatx4 wa, wb;
        fx_w8(ws[wid], 0, wa, wb);
        if constexpr (MODE == 2 || MODE == 3) fx_loadQ(vb, vt, loff, DX_Q);
        if constexpr (MODE >= 3) {
            for (int j0 = 0; j0 < n; j0 += 2 * DX_Q) {
                if constexpr (MODE == 4) fx_loadQ(vb, vt, loff, j0 + DX_Q);
#pragma unroll
                for (int g8 = 0; g8 < DX_Q / 8; g8++) fx8_fast(acc, va[g8], wa, wb);
                if constexpr (MODE == 4) fx_loadQ(va, vt, loff, j0 + 2 * DX_Q);
#pragma unroll
                for (int g8 = 0; g8 < DX_Q / 8; g8++) fx8_fast(acc, vb[g8], wa, wb);
            }
        } else if constexpr (MODE == 5) {
            for (int j0 = 0; j0 < n; j0 += 2 * DX_Q) {
                fx_loadQ(vb, vt, loff, j0 + DX_Q);
                fx_step1_lds_m(va, j0, ws[wid], (unsigned long long)__builtin_amdgcn_readfirstlane((int)flags) |
                               ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(flags >> 32)) << 32), acc, wa, wb);
                fx_loadQ(va, vt, loff, j0 + 2 * DX_Q);
                fx_step1_lds_m(vb, j0 + DX_Q, ws[wid], 0ull, acc, wa, wb);
            }
        } else
        for (int j0 = 0; j0 < n; j0 += 2 * DX_Q) {
            if constexpr (MODE < 2) fx_loadQ(vb, vt, loff, j0 + DX_Q);
            fx_step1_lds(va, j0, ws[wid], flags, acc, wa, wb);
            if constexpr (MODE < 2) fx_loadQ(va, vt, loff, j0 + 2 * DX_Q);
            fx_step1_lds(vb, j0 + DX_Q, ws[wid], flags, acc, wa, wb);
        }
    }
    const long long t1 = clock64();
    if (lane == 0) cyc[gw] = t1 - t0;
    out[gw * 64 + lane] = __builtin_bit_cast(uint16_t, acc);
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0, wpb = argc > 2 ? atoi(argv[2]) : 4;
    const unsigned long long flags = argc > 3 ? strtoull(argv[3], nullptr, 0) : 0ull;   // runtime: the slow path's code is present
    const int n = 1370, nwaves = 32, blocks = nwaves / wpb;
    uint16_t *vt, *o;
    float *w;
    long long *c;
    const size_t vbytes = (size_t)nwaves * 1024 * (DX_KC / 8 + 64) * 2;
    (void)hipMalloc(&vt, vbytes);
    (void)hipMalloc(&w, DX_KC / DX_B * FX_ST * 4);
    (void)hipMalloc(&o, nwaves * 64 * 2);
    (void)hipMalloc(&c, nwaves * 8);
    (void)hipMemset(vt, 0x31, vbytes);
    static float hw[DX_KC / DX_B * FX_ST];
    for (auto &x : hw) x = 0.5f;
    (void)hipMemcpy(w, hw, sizeof hw, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) {
        if (mode == 0) hipLaunchKernelGGL(chain_k<0>, dim3(blocks), dim3(64 * wpb), 0, 0, vt, w, n, c, o, flags);
        if (mode == 1) hipLaunchKernelGGL(chain_k<1>, dim3(blocks), dim3(64 * wpb), 0, 0, vt, w, n, c, o, flags);
        if (mode == 2) hipLaunchKernelGGL(chain_k<2>, dim3(blocks), dim3(64 * wpb), 0, 0, vt, w, n, c, o, flags);
        if (mode == 3) hipLaunchKernelGGL(chain_k<3>, dim3(blocks), dim3(64 * wpb), 0, 0, vt, w, n, c, o, flags);
        if (mode == 4) hipLaunchKernelGGL(chain_k<4>, dim3(blocks), dim3(64 * wpb), 0, 0, vt, w, n, c, o, flags);
        if (mode == 5) hipLaunchKernelGGL(chain_k<5>, dim3(blocks), dim3(64 * wpb), 0, 0, vt, w, n, c, o, flags);
        (void)hipDeviceSynchronize();
    }
    long long hc[32];
    (void)hipMemcpy(hc, c, sizeof hc, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nwaves; i++) s += hc[i];
    printf("mode %d  waves/wg %d  %.2f cycles/key\n", mode, wpb, s / nwaves / n);
    return 0;
}
