// Micro-benchmark of the decode chain variants on 32 waves (8 workgroups of
// 4, as the batch-1 fused launch's chain role), n keys of random scores:
//   mode 0: fx_weights_reg + fx_chain1 (fa_exact.hip's decode chain: all the
//           weights of the chunk first, 32 keys a lane, v_readlane per key)
//   mode 3: fxp_chain_w on mode 0's weights (the split-weights chain of the fused launch)
//   mode 1: fxp_chain (fx_pipe.h: weights one 64-key buffer ahead, lane = key,
//           SGPR weights by v_readlane inside the group blocks)
// Prints cycles per key (clock64 around the chain, mean and max over waves),
// and checks mode 1's accumulators against mode 0's bit for bit.
// usage: chain_pipe [n] [sigma] [warm: V^T pulled into L2 before the clock, default 1]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define FXP_TRACE
#include "../../qwen3-asr.cpp_amd/csrc/fx_chain.h"
#include "../../qwen3-asr.cpp_amd/csrc/fx_decode.h"
#include "../../qwen3-asr.cpp_amd/csrc/fx_pipe.h"

using namespace qasr;

#define NW 32
#define KMAX 2048
#define VBLK (KMAX / 8 + 64)

struct FxpW {   // given weights in memory
    const float *w;
    int n;
    __device__ __forceinline__ float issue(int j0) const {
        const int j = j0 + (int)(threadIdx.x & 63);
        return w[j < n ? j : 0];
    }
    __device__ __forceinline__ float take(float v, int j0) const { return j0 + (int)(threadIdx.x & 63) < n ? v : 0.0f; }
};

template <int MODE>
__global__ __launch_bounds__(256) void chain_k(const uint16_t *vt_all, const float *sc_all, int n, long long *cyc, uint16_t *out,
                                               float *sout, int warm, float *wout) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int gw = blockIdx.x * 4 + wid;
    const uint16_t *vt = vt_all + (long)gw * 1024 * VBLK;
    const float *sc = sc_all + (long)gw * KMAX;
    const int loff = 8 * lane, lastb = (n - 1) >> 3;
    f16 acc = 0;
    float S = 0.0f;
    if (warm) {   // the wave's V^T rows -> L2 first (the fused launch pulls them while the scores are computed)
        u32x4 t = {0, 0, 0, 0};
        for (int kb = 0; kb <= lastb; kb++) t += *(const u32x4 *)(vt + (long)kb * 1024 + loff);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(t));
    }
    __syncthreads();
    const long long t0 = clock64();
    if constexpr (MODE == 0) {
        float w[DX_B], wl, M = -INFINITY;
        unsigned long long flags;
        uint32_t kb;
        S = fx_weights_reg([&](int j) { return sc[j]; }, n, M, w, flags, wl, &kb);
#pragma unroll
        for (int i = 0; i < DX_B; i++) wout[gw * KMAX + lane * DX_B + i] = w[i];   // (mode 3's given weights)
        fx_chain1(vt, loff, 0, n, lastb, w, flags, kb, acc);
    } else if constexpr (MODE == 1) {
        float wlast;
        S = fxp_chain(FxpScores{sc, n}, vt, loff, n, lastb, acc, wlast);
    } else if constexpr (MODE == 2) {   // timing only: every V^T load reads key block 0 (cache-hot), the chain's instruction stream unchanged
        float wlast;
        S = fxp_chain(FxpScores{sc, n}, vt, loff, n, 0, acc, wlast);
    } else {   // fxp_chain_w on mode 0's weights (the split-weights chain), V^T as mode 1
        float wlast;
        fxp_chain_w(FxpW{wout + gw * KMAX, n}, vt, loff, n, lastb, acc, wlast);
    }
    const long long t1 = clock64();
    if (lane == 0) cyc[gw] = t1 - t0;
    out[gw * 64 + lane] = __builtin_bit_cast(uint16_t, acc);
    if (lane == 0) sout[gw] = S;
}

static uint16_t f2h_host(float f) {
    _Float16 h = (_Float16)f;
    uint16_t u;
    memcpy(&u, &h, 2);
    return u;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1370;
    const float sigma = argc > 2 ? atof(argv[2]) : 2.0f;
    const int warm = argc > 3 ? atoi(argv[3]) : 1;
    const size_t vn = (size_t)NW * 1024 * VBLK;
    uint16_t *hv = (uint16_t *)malloc(vn * 2);
    float *hs = (float *)malloc((size_t)NW * KMAX * 4);
    srand(7);
    auto gauss = []() {
        double u1 = (rand() + 1.0) / (RAND_MAX + 2.0), u2 = (rand() + 1.0) / (RAND_MAX + 2.0);
        return sqrt(-2 * log(u1)) * cos(6.283185307179586 * u2);
    };
    for (size_t i = 0; i < vn; i++) hv[i] = f2h_host((float)gauss());
    for (int i = 0; i < NW * KMAX; i++) hs[i] = (float)(sigma * gauss());
    uint16_t *vt, *o0, *o1, *o2, *o3;
    float *wts;
    float *sc, *s0, *s1, *s2;
    long long *c;
    (void)hipMalloc(&vt, vn * 2);
    (void)hipMalloc(&sc, (size_t)NW * KMAX * 4);
    (void)hipMalloc(&o0, NW * 64 * 2);
    (void)hipMalloc(&o1, NW * 64 * 2);
    (void)hipMalloc(&o2, NW * 64 * 2);
    (void)hipMalloc(&o3, NW * 64 * 2);
    (void)hipMalloc(&wts, (size_t)NW * KMAX * 4);
    (void)hipMalloc(&s0, NW * 4);
    (void)hipMalloc(&s1, NW * 4);
    (void)hipMalloc(&s2, NW * 4);
    (void)hipMalloc(&c, NW * 8);
    (void)hipMemcpy(vt, hv, vn * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(sc, hs, (size_t)NW * KMAX * 4, hipMemcpyHostToDevice);
    long long hc[NW];
    for (int mode = 0; mode < 4; mode++) {
        double best = 1e30, bmax = 0;
        for (int rep = 0; rep < 5; rep++) {
            if (mode == 0) hipLaunchKernelGGL(chain_k<0>, dim3(NW / 4), dim3(256), 0, 0, vt, sc, n, c, o0, s0, warm, wts);
            else if (mode == 1) hipLaunchKernelGGL(chain_k<1>, dim3(NW / 4), dim3(256), 0, 0, vt, sc, n, c, o1, s1, warm, wts);
            else if (mode == 2) hipLaunchKernelGGL(chain_k<2>, dim3(NW / 4), dim3(256), 0, 0, vt, sc, n, c, o2, s2, warm, wts);
            else hipLaunchKernelGGL(chain_k<3>, dim3(NW / 4), dim3(256), 0, 0, vt, sc, n, c, o3, s2, warm, wts);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(hc, c, sizeof hc, hipMemcpyDeviceToHost);
            double s = 0, mx = 0;
            for (int i = 0; i < NW; i++) {
                s += hc[i];
                mx = hc[i] > mx ? hc[i] : mx;
            }
            if (s / NW < best) {
                best = s / NW;
                bmax = mx;
            }
        }
        printf("mode %d  n %d  sigma %.1f  warm %d  %.2f cycles/key (max wave %.2f)\n", mode, n, sigma, warm, best / n, bmax / n);
    }
    {   // FXP_TRACE: wave 0 of workgroup 0, summed over all launches of modes 1 and 2
        unsigned long long tr[4];
        (void)hipMemcpyFromSymbol(tr, HIP_SYMBOL(fxp_trace), sizeof tr);
        printf("trace (wave 0, modes 1+2, 5 reps each): weights %.1f, chain %.1f cycles a key\n", tr[0] / 10.0 / n, tr[1] / 10.0 / n);
    }
    uint16_t h0[NW * 64], h1[NW * 64];
    float hs0[NW], hs1[NW];
    (void)hipMemcpy(h0, o0, sizeof h0, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h1, o1, sizeof h1, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hs0, s0, sizeof hs0, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hs1, s1, sizeof hs1, hipMemcpyDeviceToHost);
    uint16_t h3[NW * 64];
    (void)hipMemcpy(h3, o3, sizeof h3, hipMemcpyDeviceToHost);
    int diff = 0, diff3 = 0;
    for (int i = 0; i < NW * 64; i++) diff += h0[i] != h1[i];
    for (int i = 0; i < NW * 64; i++) diff3 += h0[i] != h3[i];
    printf("given-weights chain (mode 3) acc mismatches %d\n", diff3);
    diff += diff3;
    double sd = 0;
    for (int i = 0; i < NW; i++) sd = fmax(sd, fabs(hs0[i] - hs1[i]) / fabs(hs0[i]));
    printf("acc mismatches %d of %d, S max rel diff %.3g\n", diff, NW * 64, sd);
    return diff != 0;
}
