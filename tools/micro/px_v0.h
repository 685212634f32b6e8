// px_v0.h -- the round-5 exact prefill attention kernel (fa_exact.hip until
// round 6), kept as the baseline of tools/micro/px_bench: per row a full
// wave's weights pass (two keys a lane, 64-lane scans), separate vs / ms
// words, a new maximum anywhere in a 16-key batch scaling every key of it,
// the partial last batch key by key, three barriers a chunk.  The round-6
// product kernel (fa_exact.hip prefill_attn_exact_kernel) gives the same bits.
// FX_STAMPS builds (tools/micro/fx_bench.hip) record its phase cycles.
// Included after fa_exact.hip.
#pragma once

namespace qasr {

// ggml_vec_scale_f16: fp16(acc * ms)
__device__ __forceinline__ half2v fx_scale2(half2v acc, float ms) {
    return __builtin_convertvector((floatx2){(float)acc.x * ms, (float)acc.y * ms}, half2v);
}
// Weights of n keys (n <= KPL * 64) of one row, one wave: src[j] = the scaled
// score (src may be sc itself), sc[j] = vs_j on return, ms[j] = ms_j (1 where no new
// maximum; a masked key (-inf) gives vs = 0, ms = 1 -- ggml skips it, and a
// zero weight leaves the fp16 accumulator unchanged); fl[b * fls] = 1 where
// batch b (FX_B keys) holds a new maximum.  M: running maximum (in/out);
// S: rescaled to the new maximum, plus this chunk's sum.
template <int KPL>
__device__ __forceinline__ void fx_weights(const float *src, float *sc, float *ms, uint32_t *fl, int fls, int n, float &M,
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
    const float Mn = fmaxf(M, lane_f(inc, 63));
    // one expf a key, branch-free (a new maximum: ms = expf(Mold - M), 0 before the first key,
    // vs = 1; any other key: vs = expf(s - M)); round 6: the per-key if / else compiled to divergent
    // blocks around each expf (tools/micro/px_bench PMC: 2.5x the chain's VALU instructions)
    bool nm = false;
    float t[KPL];   // this chunk's S terms expf(s - Mn)
#pragma unroll
    for (int i = 0; i < KPL; i++) {
        const int j = lane * KPL + i;
        const float s = v[i];
        const bool gt = s > Mp;
        const float e = expf(gt ? Mp - s : s - Mp);
        const float m1 = gt ? e : 1.0f, w = gt ? 1.0f : (s != -INFINITY ? e : 0.0f);
        Mp = fmaxf(Mp, s);
        nm = nm || gt;
        if (j < n) {
            sc[j] = w;
            ms[j] = m1;
        }
        // where the running maximum after this key is already the chunk's, expf(s - Mn) is the weight
        // just computed (the same operands: w, or 1 = expf(0) at the maximum itself); the others
        // (keys before a later new maximum, mostly the first chunks of a row) take their own expf
        t[i] = s == -INFINITY ? 0.0f : w;
        if (Mp != Mn && s != -INFINITY) t[i] = expf(s - Mn);
    }
    float ps = 0.0f;
#pragma unroll
    for (int i = 0; i < KPL; i++) ps += t[i];
    ps = wave_sum(ps);
    // (S * expf(0) = S exactly: no rescale when the chunk held no new maximum)
    S = (M == -INFINITY ? 0.0f : M == Mn ? S : S * expf(M - Mn)) + ps;
    M = Mn;
    constexpr int LPB = FX_B / KPL;   // lanes per batch
    const unsigned long long bal = __ballot(nm);
    if (lane % LPB == 0 && lane * KPL < n) {
        const unsigned long long grp = (bal >> lane) & ((1ull << LPB) - 1ull);
        fl[(lane / LPB) * fls] = grp != 0ull;
    }
}

// One full batch of FX_B keys for R rows, two dimensions per lane: v[i] = the
// lane's V dword of key j0 + i; row r's weights at vs / ms + r * ld + j0.
// Rows whose bit is set in SCALE hold a new maximum in the batch and scale
// every key of it (ggml_vec_scale_f16 runs only on a new maximum, but ms = 1
// is exact: an fp16 value times 1, rounded to fp16); the others take three
// VALU instructions per key.
template <int R, int SCALE>
__device__ __forceinline__ void fx_body2(const uint32_t *v, const float *vs, const float *ms, int ld, int j0, half2v *acc) {
#pragma unroll
    for (int i = 0; i < FX_B; i++)
#pragma unroll
        for (int r = 0; r < R; r++) {
            if constexpr (SCALE != 0)
                if ((SCALE >> r) & 1) acc[r] = fx_scale2(acc[r], ms[r * ld + j0 + i]);
            acc[r] = fx_mad2(acc[r], v[i], vs[r * ld + j0 + i]);
        }
}
template <int R>
__device__ __forceinline__ void fx_batch2(const uint32_t *v, const float *vs, const float *ms, int ld, int j0, int nb,
                                          uint32_t mask, half2v *acc) {
    static_assert(R == 2, "row-mask dispatch written for two rows a wave");
    if (nb == FX_B) {
        switch (mask) {   // uniform
        case 0: fx_body2<R, 0>(v, vs, ms, ld, j0, acc); break;
        case 1: fx_body2<R, 1>(v, vs, ms, ld, j0, acc); break;
        case 2: fx_body2<R, 2>(v, vs, ms, ld, j0, acc); break;
        default: fx_body2<R, 3>(v, vs, ms, ld, j0, acc); break;
        }
    } else {   // the chunk's partial last batch
#pragma unroll
        for (int i = 0; i < FX_B; i++) {
            if (i < nb) {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    acc[r] = fx_scale2(acc[r], ms[r * ld + j0 + i]);
                    acc[r] = fx_mad2(acc[r], v[i], vs[r * ld + j0 + i]);
                }
            }
        }
    }
}
// the chain over keys [0, n) of a chunk for R rows, V from the chunk's LDS
// image (vl = this lane's dword of key 0, 64 dwords per key); row r's batch
// flags at fl[b * PX_ROWS + r]
template <int R>
__device__ __forceinline__ void fx_chain2(const uint32_t *vl, int n, const float *vs, const float *ms, int ld,
                                          const uint32_t *fl, half2v *acc) {
    for (int j0 = 0; j0 < n; j0 += FX_B) {
        uint32_t v[FX_B];
#pragma unroll
        for (int i = 0; i < FX_B; i++) v[i] = vl[(j0 + i) * 64];   // rows past n: staged padding, unused
        uint32_t mask = 0;
#pragma unroll
        for (int r = 0; r < R; r++) mask |= (fl[(j0 / FX_B) * PX_ROWS + r] ? 1u : 0u) << r;
        fx_batch2<R>(v, vs, ms, ld, j0, min(FX_B, n - j0), __builtin_amdgcn_readfirstlane(mask), acc);
    }
}

// FX_STAMPS (tools/micro/fx_bench.hip only): per-workgroup phase cycles of the
// prefill kernel, wave 0: [start, end, scores, weights, chain, chunks]
#ifdef FX_STAMPS
__device__ unsigned long long fx_stamps[1 << 16][8];
#define FX_CLK(v) const unsigned long long v = clock64()
#define FX_ADD(i, d) tsum[i] += (d)
#else
#define FX_CLK(v)
#define FX_ADD(i, d)
#endif


template <bool F32S>   // fp32 Q / K scores (the aligner)
__global__ __launch_bounds__(64 * PX_W, PX_MINW) void prefill_attn_exact_r5_kernel(PrefillAttnArgs a) {
    __shared__ __attribute__((aligned(16))) float sc[PX_ROWS][PX_SCS];   // scores, then vs
    __shared__ __attribute__((aligned(16))) float msw[PX_ROWS][PX_SCS];
    __shared__ __attribute__((aligned(16))) uint32_t fl[PX_KC / FX_B][PX_ROWS];
    __shared__ __attribute__((aligned(16))) uint32_t vsh[PX_KC * 64];    // the chunk's V rows
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
    // B fragment of query column ql (row q0 + ql; zero past the sequence)
    half8 qf[4];
    const bool qv = q0 + ql < L;
#pragma unroll
    for (int s = 0; s < 4; s++)
        qf[s] = qv ? *(const half8 *)(a.q + (long)(row0 + q0 + ql) * QD + h * 128 + 32 * s + 8 * g) : half8{};
    // a chunk after P0 cached tokens (TextDecoder::forward at n_past > 0): row t
    // at position P0 + t, keys 0 .. P0 + L - 1 (the aligner's fp32 K rows: P0 = 0)
    const int P0 = a.seq_pos0 ? a.seq_pos0[sq] : 0;
    const int lim = qv ? P0 + q0 + ql : -1;   // causal: keys <= the query's position
    const int kend = min(P0 + L, P0 + q0 + PX_ROWS);
    const int r0 = PX_R * wid;                                     // this wave's first row
    const int wlast = min(P0 + L - 1, P0 + q0 + r0 + PX_R - 1);    // its last key (its longest row)
    float M[PX_R], S[PX_R];
    half2v acc[PX_R];
#pragma unroll
    for (int r = 0; r < PX_R; r++) {
        M[r] = -INFINITY;
        S[r] = 0.0f;
        acc[r] = half2v{0, 0};
    }
#ifdef FX_STAMPS
    unsigned long long tsum[4] = {0, 0, 0, 0};
    FX_CLK(tk0);
#endif
    for (int c0 = 0; c0 < kend; c0 += PX_KC) {
        const int n = min(PX_KC, kend - c0);
        __syncthreads();   // the previous chunk's chains are done with sc / msw / fl / vsh
        FX_CLK(ta);
        // V rows c0 .. c0 + PX_KC - 1 -> LDS: 1 KiB (4 rows) per wave-instruction
#pragma unroll
        for (int it = wid; it < PX_KC / 4; it += PX_W)
            __builtin_amdgcn_global_load_lds((glb_void *)(vc + (long)(c0 + 4 * it + (lane >> 4)) * 128 + 8 * (lane & 15)),
                                             (lds_void *)(vsh + it * 256), 16, 0, 0);
        // (1) scores: 16-key tile t = wid
        if constexpr (F32S) {   // fp32 Q and K (the aligner): v_mfma_f32_16x16x4_f32, exact fp32 products
            const int t = wid;
            if (t * 16 < n) {
                // lane (row r = lane & 15, group g): dims 32 g .. 32 g + 31 of key r / query r
                // (any split of the 128 dims works if A and B use the same one)
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
                for (int kk = 0; kk < 32; kk += 2) {   // two accumulators: the 40-cycle dependent latency
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
            const int t = wid;
            const int key = min(c0 + t * 16 + ql, kend - 1);
            half8 kf[4];
#pragma unroll
            for (int s = 0; s < 4; s++) kf[s] = *(const half8 *)(kc + (long)key * 128 + 32 * s + 8 * g);
            if (t * 16 < n) {
                floatx4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 4; s++) sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], qf[s], sacc, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 4; i++) {   // C row = key 4g + i of the tile, column = query ql
                    const int k = c0 + t * 16 + 4 * g + i;
                    sc[ql][t * 16 + 4 * g + i] = k <= lim ? sacc[i] * a.scale : -INFINITY;
                }
            }
        }
        __syncthreads();
        FX_CLK(tb);
        FX_ADD(0, tb - ta);
        // (2) weights of the wave's rows
#pragma unroll
        for (int r = 0; r < PX_R; r++)
            fx_weights<PX_KC / 64>(sc[r0 + r], sc[r0 + r], msw[r0 + r], &fl[0][r0 + r], PX_ROWS, n, M[r], S[r]);
        __syncthreads();   // (the V image has landed: the barrier drains the LDS-DMA)
        FX_CLK(tc);
        FX_ADD(1, tc - tb);
        // (3) the chain, up to the wave's longest row (a shorter row sees zero weights)
        const int nw = min(n, wlast + 1 - c0);
        if (nw > 0) fx_chain2<PX_R>(vsh + lane, nw, sc[r0], msw[r0], PX_SCS, &fl[0][r0], acc);
        FX_CLK(td);
        FX_ADD(2, td - tc);
        FX_ADD(3, 1);
    }
#ifdef FX_STAMPS
    if (tid == 0) {
        unsigned long long *st = fx_stamps[blockIdx.x + gridDim.x * blockIdx.y];
        st[0] = tk0;
        st[1] = clock64();
        for (int i = 0; i < 4; i++) st[2 + i] = tsum[i];
        st[6] = q0;
    }
#endif
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
