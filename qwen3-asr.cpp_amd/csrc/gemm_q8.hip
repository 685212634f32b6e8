// gemm_q8.hip -- the Q8_0 block GEMM of the encoder / prefill projections
// (split from gemm.hip: built with -mllvm -amdgpu-mfma-vgpr-form=1 so the int8
// MFMA results land in VGPRs; in AGPRs every result came back through four
// v_accvgpr_read_b32, 12 VALU per MFMA where the block scaling needs 8).
#include "gemm_epi.h"

namespace qasr {

// ================================================================ Q8_0 GEMM
// ggml_mul_mat(W Q8_0, X) = per 32-wide K block: exact int8 dot (here one
// v_mfma_i32_16x16x32_i8 with a zero accumulator), converted to fp32 and
// fma'd with d_w * d_x into the fp32 accumulator (ggml_vec_dot_q8_0_q8_0:
// sumf += (d_x * d_y) * sumi).  A and W are staged as int8 rows of KS blocks
// (row stride KS*32+16 B: the 8-byte fragment reads of 16 lanes hit distinct
// bank pairs), their block scales as fp32 beside them.

template <int BM, int BN, int KS, int EPI>
__global__ __launch_bounds__(256) void gemm_q8_kernel(GemmArgs g) {
    constexpr int FM = BM / 32, FN = BN / 32;
    constexpr int ROWS = BM + BN;
    constexpr int RB = KS * 32 + 16;           // LDS bytes per row per stage
    constexpr int NCH = ROWS * KS * 2;         // 16-byte chunks per stage
    constexpr int CPT = (NCH + 255) / 256;
    static_assert(ROWS <= 256, "one scale row per thread");
    __shared__ __attribute__((aligned(16))) int8_t sq[2][ROWS * RB];
    __shared__ __attribute__((aligned(16))) float ssc[2][KS][ROWS];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int M = g.M, K = g.K, nbw = K / 32;

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    u32x4 stage[CPT];
    float sreg[KS];
    auto gload = [&](int k0) {
#pragma unroll
        for (int t = 0; t < CPT; t++) {
            const int c = tid + t * 256;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (c < NCH) {
                const int r = c / (KS * 2), q = c - r * (KS * 2);
                const int k = k0 + q * 16;
                if (r < BM) {
                    const int row = m0 + r;
                    if (row < M) v = *(const u32x4 *)(g.Aq + (long)row * g.lda + k);
                } else {
                    v = *(const u32x4 *)(g.Wq + (long)(n0 + r - BM) * g.ldw + k);
                }
            }
            stage[t] = v;
        }
        if (tid < ROWS) {
            const int kb = k0 / 32;
            if (tid < BM) {
                const int row = m0 + tid;
#pragma unroll
                for (int u = 0; u < KS; u++) sreg[u] = row < M ? g.Ad[(long)row * g.ldad + kb + u] : 0.0f;
            } else {
                const uint16_t *wd = g.Wd + (long)(n0 + tid - BM) * nbw + kb;
#pragma unroll
                for (int u = 0; u < KS; u++) sreg[u] = u16_to_f(wd[u]);
            }
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int t = 0; t < CPT; t++) {
            const int c = tid + t * 256;
            if (c < NCH) {
                const int r = c / (KS * 2), q = c - r * (KS * 2);
                *(u32x4 *)(&sq[buf][r * RB + q * 16]) = stage[t];
            }
        }
        if (tid < ROWS)
#pragma unroll
            for (int u = 0; u < KS; u++) ssc[buf][u][tid] = sreg[u];
    };

    const int nk = K / (32 * KS);
    gload(0);
    sstore(0);
    __syncthreads();
    const int kg = lane >> 4;
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * 32 * KS);
        // (not unrolled: unrolled, every block's fragments and scales were loaded
        // up front, 188 VGPRs and 2 waves a SIMD; rolled 100-120 VGPRs, 4 waves)
#pragma unroll 1
        for (int u = 0; u < KS; u++) {
            long af[FM], bf[FN];
            floatx4 sa[FM];
            float sb[FN];
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const int r = wr * (BM / 2) + i * 16 + (lane & 15);
                af[i] = *(const long *)(&sq[cur][r * RB + u * 32 + kg * 8]);
                sa[i] = *(const floatx4 *)(&ssc[cur][u][wr * (BM / 2) + i * 16 + 4 * kg]);
            }
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int r = BM + wc * (BN / 2) + j * 16 + (lane & 15);
                bf[j] = *(const long *)(&sq[cur][r * RB + u * 32 + kg * 8]);
                sb[j] = ssc[cur][u][r];
            }
            // software-pipelined: fragment f's MFMA is issued, then f - 1's result
            // scaled, with the order pinned (sched_barrier) -- left alone the
            // scheduler issued all FM * FN MFMAs first, so their results went to
            // AGPRs and every one came back by 4 v_accvgpr_read (12 VALU per MFMA
            // where the scaling needs 8); the same operations, so the same bits
            intx4 cp = __builtin_amdgcn_mfma_i32_16x16x32_i8(af[0], bf[0], intx4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
            for (int f = 1; f <= FM * FN; f++) {
                intx4 cn = cp;
                if (f < FM * FN) cn = __builtin_amdgcn_mfma_i32_16x16x32_i8(af[f / FN], bf[f % FN], intx4{0, 0, 0, 0}, 0, 0, 0);
                q8_scale_acc(acc[(f - 1) / FN][(f - 1) % FN], sb[(f - 1) % FN], sa[(f - 1) / FN], cp);
                __builtin_amdgcn_sched_barrier(0);
                cp = cn;
            }
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }
    gemm_epilogue<BM, BN, EPI>(g, acc, m0, n0, wr, wc, lane);
}

template <int BM, int BN, int KS, int EPI>
static void run_gemm_q8(const GemmArgs &g, hipStream_t s) {
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    hipLaunchKernelGGL((gemm_q8_kernel<BM, BN, KS, EPI>), grid, dim3(256), 0, s, g);
}

template <int EPI>
static void dispatch_q8(const GemmArgs &g, hipStream_t s) {
    const bool big = g.M >= 2048 && g.N % 128 == 0;
    if (g.K % 128 == 0) {
        // large M: 128 x 64 tiles (4 x 2 fragments a wave).  With 128 x 128 the 64
        // fp32 accumulators a wave did not fit beside the MFMA results and every
        // block's scaling shuttled them through AGPRs (~10 v_accvgpr moves per
        // MFMA on top of the 8 scaling ops): configs[2] prefill 152.6 -> 121.6 ms,
        // encode 80.6 -> 64.3 (64 x 64: 130.3 / 67.4, 64 x 128: 122.5 / 65.2;
        // 128 x 128 with 128-wide K stages: 306 ms, one workgroup a CU)
        // (128 x 64 with 128-wide K stages: 162.1 ms; 96 x 64: 129.7)
        if (big && g.N % 64 == 0) run_gemm_q8<128, 64, 2, EPI>(g, s);
        else if (big) run_gemm_q8<128, 128, 2, EPI>(g, s);
        else run_gemm_q8<64, 64, 4, EPI>(g, s);
    } else {
        run_gemm_q8<64, 64, 1, EPI>(g, s);
    }
}

void launch_gemm_q8(int epi, const GemmArgs &g, hipStream_t s) {
    if (g.M <= 0) return;
    switch (epi) {
        case EPI_F32: dispatch_q8<EPI_F32>(g, s); break;
        case EPI_GELU_F16: dispatch_q8<EPI_GELU_F16>(g, s); break;
        case EPI_SWIGLU_F32: dispatch_q8<EPI_SWIGLU_F32>(g, s); break;
        default: break;
    }
}

}  // namespace qasr
