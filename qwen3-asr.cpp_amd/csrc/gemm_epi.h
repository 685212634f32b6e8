// gemm_epi.h -- the tiled GEMMs' shared pieces: the conv chunk lookup and the
// per-element epilogue (+bias, +residual, GELU / SwiGLU / fp16 / argmax
// outputs) over the v_mfma_*_16x16x* C layout.  Used by gemm.hip (fp16) and
// gemm_q8.hip (Q8_0), which is compiled on its own for its MFMA register form.
#pragma once
#include <type_traits>

#include "dev_common.h"
#include "kernels.h"

namespace qasr {

__device__ __forceinline__ int find_chunk(const int *__restrict__ starts, int n, int r) {
    int lo = 0, hi = n - 1;   // largest c with starts[c] <= r
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (starts[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ float silu_f(float g) { return g / (1.0f + expf(-g)); }

// ------------------------------------------------------------ epilogue
// acc[i][j] holds rows m0 + wr*BM/2 + 16i + 4(lane>>4) + r, column
// n0 + wc*BN/WNW + 16j + (lane&15) (v_mfma_*_16x16x* C layout; WNW waves along N)
template <int BM, int BN, int EPI, int WNW = 2>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs &g, floatx4 (&acc)[BM / 32][BN / (16 * WNW)], int m0, int n0, int wr,
                                              int wc, int lane) {
    constexpr int FM = BM / 32, FN = BN / (16 * WNW);
    const int M = g.M;
    const int rbase = m0 + wr * (BM / 2) + 4 * (lane >> 4);
    const int cbase = n0 + wc * (BN / WNW) + (lane & 15);
    if constexpr (EPI == EPI_SWIGLU_F16 || EPI == EPI_SWIGLU_F32) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int p = 0; p < FN / 2; p++) {
                const int ocol = (n0 + wc * (BN / WNW)) / 2 + p * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = rbase + i * 16 + r;
                    if (row < M) {
                        const float gt = acc[i][2 * p][r], up = acc[i][2 * p + 1][r];
                        const float v = silu_f(gt) * up;
                        if constexpr (EPI == EPI_SWIGLU_F32) g.out_f32[(long)row * g.ldo + ocol] = v;
                        else g.out_f16[(long)row * g.ldo16 + ocol] = f_to_u16(v);
                    }
                }
            }
    } else if constexpr (EPI == EPI_ARGMAX) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = rbase + i * 16 + r;
                unsigned long long best = 0ull;
#pragma unroll
                for (int j = 0; j < FN; j++) {
                    const int col = cbase + j * 16;
                    const float v = acc[i][j][r];
                    if (row < M && g.out_f32) g.out_f32[(long)row * g.ldo + col] = v;
                    const unsigned long long key = (g.n_valid == 0 || col < g.n_valid) ? argmax_key(v, col) : 0ull;
                    best = key > best ? key : best;
                }
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const unsigned long long other = __shfl_xor(best, o, 64);
                    best = other > best ? other : best;
                }
                if (row < M && (lane & 15) == 0) atomicMax(g.amax + row, best);
            }
    } else {
        // Every load the values need (bias at entry; residual / PE / GELU table one
        // 16-row block at a time) is issued before the stores that precede its use: a
        // load behind a store makes its use wait for that store's write to complete, and
        // the per-element form compiled to vmcnt(0) ahead of every store (round 6, as
        // gemm8p.h's epilogue).
        float bcol[FN];
#pragma unroll
        for (int j = 0; j < FN; j++) bcol[j] = g.bias ? g.bias[cbase + j * 16] : 0.0f;
        auto stores = [&](int i, const float (&v)[FN][4]) {
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int col = cbase + j * 16;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = rbase + i * 16 + r;
                    if (row >= M) continue;
                    if constexpr (EPI == EPI_GELU_F16 || EPI == EPI_F16) g.out_f16[(long)row * g.ldo16 + col] = (uint16_t)__float_as_uint(v[j][r]);
                    else g.out_f32[(long)row * g.ldo + col] = v[j][r];
                }
            }
        };
#pragma unroll
        for (int i = 0; i < FM; i++) {
            float v[FN][4];
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int r = 0; r < 4; r++) v[j][r] = g.bias ? fadd_rn(acc[i][j][r], bcol[j]) : acc[i][j][r];
            if constexpr (EPI == EPI_GELU_F16 || EPI == EPI_F16) {
                // fp16 bits carried in the float array (bit cast) up to the stores
#pragma unroll
                for (int j = 0; j < FN; j++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float x = v[j][r];
                        const uint32_t b16 = f_to_u16(x);
                        uint32_t h = b16;
                        if constexpr (EPI == EPI_GELU_F16) {
                            // gelu_lut's selects as bit masks (a select on a loaded value
                            // becomes a branch around the load); the table read clamped into
                            // the table for every value
                            const uint32_t t = g.gelu[b16];
                            const uint32_t hi = 0u - (uint32_t)(x >= 10.0f), lo = 0u - (uint32_t)(x <= -10.0f);
                            h = ((t & ~hi) | (b16 & hi)) & ~lo;
                        }
                        v[j][r] = __uint_as_float(h);
                    }
                stores(i, v);
            } else if (g.pe || g.res) {
                float pv[FN][4], rv[FN][4];
#pragma unroll
                for (int j = 0; j < FN; j++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = min(rbase + i * 16 + r, M - 1), col = cbase + j * 16;
                        pv[j][r] = g.pe ? g.pe[(long)g.pe_pos[row] * g.N + col] : 0.0f;
                        rv[j][r] = g.res ? g.res[(long)row * g.ldr + col] : 0.0f;
                    }
#pragma unroll
                for (int j = 0; j < FN; j++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        if (g.pe) v[j][r] = fadd_rn(v[j][r], pv[j][r]);
                        if (g.res) v[j][r] = fadd_rn(v[j][r], rv[j][r]);
                    }
                stores(i, v);
            } else {
                stores(i, v);
            }
        }
    }
}

}  // namespace qasr
