// px_v3.h -- round-6 experiment, measured and NOT taken:
// fa_exact.hip's exact prefill attention rescheduled -- the next chunk's K
// fragments (registers) and V image (LDS-DMA into a double buffer) requested
// right after the score MFMAs, Q rows in LDS, two barriers a chunk instead of
// three, weights sign-encoded in the score rows, per-batch 16-bit new-maximum
// masks so only those keys take the scale (v_fma_mix_f32 with a neg(0) addend),
// and the diagonal chunk's partial batch run as a full body with v = -0 past
// the wave's last key.  Bit-identical to the product kernel on every
// tools/micro/px_bench case, but not faster: 2778 vs 2622 us at 128 x 405
// (alternating runs, one box), 2624 with FX_B = 8; PMC: VALU instructions
// 1.19e9 vs 1.27e9, SALU +40 %, branches x2 (profiles/r6/prefill_attn.txt).
// Included by tools/micro/px_bench.hip after fa_exact.hip.
#pragma once

namespace qasr {

template <int KPL, bool ENC = true>
__device__ __forceinline__ void fx_weights_enc(const float *src, float *sc, float *ms, uint32_t *fl, int fls, int n, float &M,
                                           float &S) {
    const int lane = threadIdx.x & 63;
    float v[KPL];
    float lm = -INFINITY;
#pragma unroll
    for (int i = 0; i < KPL; i++) {   // independent loads (src: LDS, or the scores in global memory)
        const int j = lane * KPL + i;
        v[i] = j < n ? src[j] : -INFINITY;
    }
#pragma unroll
    for (int i = 0; i < KPL; i++) lm = fmaxf(lm, v[i]);
    const float inc = wave_scan_max(lm);   // inclusive prefix maximum over the lanes
    float Mp = fmaxf(M, dpp_ninf<0x138, 0xF>(inc));   // wave_shr:1 -> the exclusive prefix (lane 0: -inf)
    bool nm = false;
    bool kmv[KPL];
#pragma unroll
    for (int i = 0; i < KPL; i++) {
        const int j = lane * KPL + i;
        const float s = v[i];
        float m1 = 1.0f, w = 0.0f;
        bool km = false;
        if (s > Mp) {   // new maximum: ms = expf(Mold - M) (0 before the first key), vs = 1
            m1 = expf(Mp - s);
            w = 1.0f;
            Mp = s;
            nm = true;
            km = true;
        } else if (s != -INFINITY) {
            w = expf(s - Mp);
        }
        kmv[i] = km && j < n;
        if (j < n) {
            if constexpr (ENC) {   // one word a key: -ms at a new maximum (vs = 1 there; -0 before the first), else vs >= 0
                sc[j] = km ? -m1 : w;
            } else {
                sc[j] = w;
                ms[j] = m1;
            }
        }
    }
    if constexpr (ENC) {   // keys past n within the chunk: weight 0 (the chain's last batch may read them)
#pragma unroll
        for (int i = 0; i < KPL; i++) {
            const int j = lane * KPL + i;
            if (j >= n && j < 64 * KPL) sc[j] = 0.0f;
        }
    }
    const float Mn = fmaxf(M, lane_f(inc, 63));
    float ps = 0.0f;
#pragma unroll
    for (int i = 0; i < KPL; i++) ps += v[i] == -INFINITY ? 0.0f : expf(v[i] - Mn);
    ps = wave_sum(ps);
    S = (M == -INFINITY ? 0.0f : S * expf(M - Mn)) + ps;
    M = Mn;
    constexpr int LPB = FX_B / KPL;   // lanes per batch
    if constexpr (ENC) {
        // fl[b * fls] = the batch's new-maximum keys as a bit mask (bit i = key 16 b + i): the chain
        // scales the accumulator exactly there (elsewhere ms = 1, an exact no-op)
        static_assert(FX_B <= 32 && LPB >= 1, "a batch's key mask in one word");
        uint32_t mb = 0;
#pragma unroll
        for (int i = 0; i < KPL; i++) {
            mb |= (kmv[i] ? 1u : 0u) << (KPL * (lane % LPB) + i);
        }
#pragma unroll
        for (int o = 1; o < LPB; o <<= 1) mb |= __shfl_xor(mb, o, 64);
        if (lane % LPB == 0 && lane * KPL < n) fl[(lane / LPB) * fls] = mb;
    } else {
        const unsigned long long bal = __ballot(nm);
        if (lane % LPB == 0 && lane * KPL < n) {
            const unsigned long long grp = (bal >> lane) & ((1ull << LPB) - 1ull);
            fl[(lane / LPB) * fls] = grp != 0ull;
        }
    }
}


// The same chain over sign-encoded weights and per-batch new-maximum masks
// (fx_weights<KPL, true>: one word a key, -ms at a new maximum where vs = 1;
// fl = a 16-bit key mask per batch and row).  ggml scales the accumulator only
// at a new maximum (ggml_vec_scale_f16), which fx_body2 did for every key of
// a batch holding one (by ms = 1 elsewhere: exact); here only the masked keys
// take the scale -- fp16(fp32(acc * ms)) as v_fma_mix_f32 with a -0 addend
// (x + -0 = x, signs of zero included) and the sign of w folded into its
// neg modifier -- and every other key the plain step, so the arithmetic is
// the same key for key.  A batch past the wave's last key (the diagonal chunk)
// runs the full body with v = -0 there: w is +0 for those keys (masked, or
// zeroed past the chunk's end), so fma(-0, +0, acc) = acc + (-0) = acc exactly.
__device__ __forceinline__ half2v fx_scale2m(half2v acc, float wneg) {   // fp16(acc * -wneg), per half
    float f0, f1;
    uint32_t a = __builtin_bit_cast(uint32_t, acc), r;
    asm("v_fma_mix_f32 %0, %2, -%3, neg(0) op_sel:[0,0,0] op_sel_hi:[1,0,0]\n\t"
        "v_fma_mix_f32 %1, %2, -%3, neg(0) op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(f0), "=&v"(f1) : "v"(a), "v"(wneg));
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(f0), "v"(f1));
    return __builtin_bit_cast(half2v, r);
}
template <int R>
__device__ __forceinline__ void fx_body2m(const uint32_t *v, const float *w, int ld, int j0, uint32_t m0, uint32_t m1, half2v *acc) {
#pragma unroll
    for (int i = 0; i < FX_B; i++)
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float wk = w[r * ld + j0 + i];
            if (((r == 0 ? m0 : m1) >> i) & 1u) {   // uniform
                acc[r] = fx_scale2m(acc[r], wk);
                acc[r] = fx_mad2(acc[r], v[i], 1.0f);
            } else {
                acc[r] = fx_mad2(acc[r], v[i], wk);
            }
        }
}
template <int R>
__device__ __forceinline__ void fx_chain2m(const uint32_t *vl, int nw, const float *w, int ld, const uint32_t *fl, half2v *acc) {
    static_assert(R == 2, "two rows a wave");
    for (int j0 = 0; j0 < nw; j0 += FX_B) {
        uint32_t v[FX_B];
#pragma unroll
        for (int i = 0; i < FX_B; i++) v[i] = vl[(j0 + i) * 64];
        if (j0 + FX_B > nw) {   // uniform: the wave's last keys
#pragma unroll
            for (int i = 0; i < FX_B; i++) v[i] = j0 + i < nw ? v[i] : 0x80008000u;
        }
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(fl[(j0 / FX_B) * PX_ROWS]);
        const uint32_t m1 = __builtin_amdgcn_readfirstlane(fl[(j0 / FX_B) * PX_ROWS + 1]);
        if ((m0 | m1) == 0u) {
#pragma unroll
            for (int i = 0; i < FX_B; i++)
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] = fx_mad2(acc[r], v[i], w[r * ld + j0 + i]);
        } else {
            fx_body2m<R>(v, w, ld, j0, m0, m1, acc);
        }
    }
}


#ifdef FX_STAMPS
#define PX3_STAMPS 1
#endif
// Round 6: the same arithmetic in a schedule that keeps the
// chain issuing.  The round-5 kernel waited, every 128-key chunk, for its K
// fragments (loaded after the chunk's first barrier) and for the V image
// (landing during the scores and weights), and synchronised three times.  Here:
//  * the next chunk's K fragments and V image are requested right after this
//    chunk's score MFMAs (K into registers, V by LDS-DMA into the other half of
//    a double-buffered image), so they land under the weights and the chain;
//  * the weights are sign-encoded in the score rows (fx_weights<.., true>: -ms
//    at a new maximum, vs elsewhere) instead of a second array, and the Q rows
//    sit in LDS (16-B chunks swizzled by row) instead of 16 VGPRs a lane, so two
//    workgroups still fit a CU (77 KiB of LDS, <= 128 VGPRs);
//  * two barriers a chunk: (1) the previous chunk's chains are done and this
//    chunk's K / V have landed, (2) the scores are in LDS; each wave then derives
//    its own rows' weights and runs their chains with no further barrier.
// Same scores (same MFMA fragments and order), same weights (same scans and
// 128-key S partition), same chain arithmetic: the outputs are bit-identical.
template <bool F32S>
__global__ __launch_bounds__(64 * PX_W, 2) void prefill_attn_exact2_kernel(PrefillAttnArgs a) {
    __shared__ __attribute__((aligned(16))) float sc[PX_ROWS][PX_SCS];        // scores, then encoded weights
    __shared__ __attribute__((aligned(16))) uint32_t fl[PX_KC / FX_B][PX_ROWS];
    __shared__ __attribute__((aligned(16))) uint32_t vsh[2][PX_KC * 64];      // chunk c's V rows in vsh[c & 1]
    __shared__ __attribute__((aligned(16))) uint16_t qsh[PX_ROWS * 128];       // Q rows, chunk ch of row r at ch ^ r
    const int sq = blockIdx.z, h = blockIdx.y;
    const int L = a.seq_len[sq];
    const int nqb = (a.max_len + PX_ROWS - 1) / PX_ROWS;
    const int q0 = (nqb - 1 - (int)blockIdx.x) * PX_ROWS;
    if (q0 >= L) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, ql = lane & 15;
    const int hk = h / (a.n_head / a.n_kv_head);
    const int row0 = a.seq_row0[sq];
    const int QD = a.n_head * 128;
    const long cbase = ((long)a.seq_slot[sq] * a.n_kv_head + hk) * a.max_ctx;
    const uint16_t *kc = a.kc + cbase * 128, *vc = a.vc + cbase * 128;
    const bool qv = q0 + ql < L;
    const int P0 = a.seq_pos0 ? a.seq_pos0[sq] : 0;
    const int lim = qv ? P0 + q0 + ql : -1;   // causal: keys <= the query's position
    const int kend = min(P0 + L, P0 + q0 + PX_ROWS);
    const int r0 = PX_R * wid;
    const int wlast = min(P0 + L - 1, P0 + q0 + r0 + PX_R - 1);
    if constexpr (!F32S) {
        if (tid < PX_ROWS * 16) {   // Q rows -> LDS (zeros past the sequence)
            const int r = tid >> 4, ch = tid & 15;
            const u32x4 v = q0 + r < L ? *(const u32x4 *)(a.q + (long)(row0 + q0 + r) * QD + h * 128 + 8 * ch) : u32x4{0u, 0u, 0u, 0u};
            *(u32x4 *)(qsh + r * 128 + ((ch ^ r) << 3)) = v;
        }
    }
    auto issue_v = [&](int c0, int b) {   // V rows c0 .. c0 + PX_KC - 1 -> vsh[b]: 1 KiB (4 rows) a wave-instruction
#pragma unroll
        for (int it = wid; it < PX_KC / 4; it += PX_W)
            __builtin_amdgcn_global_load_lds((glb_void *)(vc + (long)(c0 + 4 * it + (lane >> 4)) * 128 + 8 * (lane & 15)),
                                             (lds_void *)(vsh[b] + it * 256), 16, 0, 0);
    };
    half8 kf[4];
    auto load_k = [&](int c0) {   // this wave's 16-key tile of the chunk at c0 (clamped: rows past kend unused)
        const int key = min(c0 + wid * 16 + ql, kend - 1);
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) kf[s4] = *(const half8 *)(kc + (long)key * 128 + 32 * s4 + 8 * g);
    };
    float M[PX_R], S[PX_R];
    half2v acc[PX_R];
#pragma unroll
    for (int r = 0; r < PX_R; r++) {
        M[r] = -INFINITY;
        S[r] = 0.0f;
        acc[r] = half2v{0, 0};
    }
    issue_v(0, 0);
    if constexpr (!F32S) load_k(0);
    int b = 0;
#ifdef FX_STAMPS
    unsigned long long tsum[6] = {0, 0, 0, 0, 0, 0}, tl = clock64();
    const unsigned long long tk0 = tl;
#define PX_MARK(i) do { const unsigned long long t_ = clock64(); tsum[i] += t_ - tl; tl = t_; } while (0)
#else
#define PX_MARK(i)
#endif
    for (int c0 = 0; c0 < kend; c0 += PX_KC, b ^= 1) {
        const int n = min(PX_KC, kend - c0);
        PX_MARK(5);
        __syncthreads();   // (1) the previous chunk's chains are done with sc / fl; this chunk's K / V (and Q) landed
        PX_MARK(0);
        const int t = wid;
        if constexpr (F32S) {   // fp32 Q and K (the aligner): v_mfma_f32_16x16x4_f32, exact fp32 products
            if (t * 16 < n) {
                const int key = min(c0 + t * 16 + ql, kend - 1);
                const float *kr = a.k32 + (long)(row0 + key) * (a.n_kv_head * 128) + hk * 128 + 32 * g;
                const float *qr = a.q32 + (long)(row0 + min(q0 + ql, L - 1)) * QD + h * 128 + 32 * g;
                float kv[32], qv2[32];
#pragma unroll
                for (int i = 0; i < 32; i += 4) {
                    *(float4 *)&kv[i] = *(const float4 *)&kr[i];
                    *(float4 *)&qv2[i] = qv ? *(const float4 *)&qr[i] : float4{0.f, 0.f, 0.f, 0.f};
                }
                floatx4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < 32; kk += 2) {
                    s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[kk], qv2[kk], s0, 0, 0, 0);
                    s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[kk + 1], qv2[kk + 1], s1, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int k = c0 + t * 16 + 4 * g + i;
                    sc[ql][t * 16 + 4 * g + i] = k <= lim ? (s0[i] + s1[i]) * a.scale : -INFINITY;
                }
            }
        } else {
            if (t * 16 < n) {
                floatx4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++) {
                    const half8 qf = *(const half8 *)(qsh + ql * 128 + (((4 * s4 + g) ^ ql) << 3));
                    sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s4], qf, sacc, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {   // C row = key 4g + i of the tile, column = query ql
                    const int k = c0 + t * 16 + 4 * g + i;
                    sc[ql][t * 16 + 4 * g + i] = k <= lim ? sacc[i] * a.scale : -INFINITY;
                }
            }
        }
        // the next chunk's K fragments and V image: requested now, needed after the next barrier (1)
        if (c0 + PX_KC < kend) {
            issue_v(c0 + PX_KC, b ^ 1);
            if constexpr (!F32S) load_k(c0 + PX_KC);
        }
        PX_MARK(1);
        __syncthreads();   // (2) every score tile of the chunk is in LDS
        PX_MARK(2);
        // the wave's rows: weights (in place, sign-encoded), then the chain up to its longest row
#pragma unroll
        for (int r = 0; r < PX_R; r++) fx_weights_enc<PX_KC / 64, true>(sc[r0 + r], sc[r0 + r], nullptr, &fl[0][r0 + r], PX_ROWS, n, M[r], S[r]);
        PX_MARK(3);
        const int nw = min(n, wlast + 1 - c0);
        if (nw > 0) fx_chain2m<PX_R>(vsh[b] + lane, nw, sc[r0], PX_SCS, &fl[0][r0], acc);
        PX_MARK(4);
    }
#ifdef FX_STAMPS
    if (lane == 0) {   // per wave: [start, end, barrier-1 wait, scores, barrier-2 wait, weights, chain, (unused)]
        unsigned long long *st = fx_stamps[((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) % 8192 * 8 + wid];
        st[0] = tk0;
        st[1] = clock64();
        for (int i = 0; i < 5; i++) st[2 + i] = tsum[i];
        st[7] = tsum[5];
    }
#endif
#undef PX_MARK
#pragma unroll
    for (int r = 0; r < PX_R; r++) {
        const int q = q0 + r0 + r;
        if (q >= L) continue;
        const float inv = S[r] == 0.0f ? 0.0f : 1.0f / S[r];
        const float o0 = (float)acc[r].x * inv, o1 = (float)acc[r].y * inv;
        const long o = (long)(row0 + q) * QD + h * 128 + 2 * lane;
        if (a.out32) {
            a.out32[o] = o0;
            a.out32[o + 1] = o1;
        } else {
            *(uint32_t *)(a.out + o) = (uint32_t)f_to_u16(o0) | ((uint32_t)f_to_u16(o1) << 16);
        }
    }
}


}  // namespace qasr
