// fx_decode.h -- the decode side of fa_exact.hip's ggml flash-attention
// numerics (text_decoder.cpp:534-540): one query row's sequential fp16 V
// chain per (head, dimension), V from the V^T cache.  Shared by
// fa_exact.hip's chain kernels (scores from global memory) and attention.hip's
// one-launch decode-batch kernel (scores kept in LDS).
#pragma once
#include "dev_common.h"
#include "fx_chain.h"
#include "kernels.h"

namespace qasr {

// ------------------------------------------------------------------- decode
// The chain for one row, one dimension per lane, V from the V^T cache (this
// lane's dimension: 8 keys per 16-B load, a wave's loads 1 KiB contiguous;
// key blocks past lastb re-read lastb, fx_loadQ).
// No LDS: each wave derives the whole chunk's weights itself, lane L holding
// keys 32 L .. 32 L + 31 in registers, and the chain takes key k's weight
// with v_readlane (an SGPR operand of v_fma_mix_f32, in the slot the mix ->
// convert dependency leaves empty).  Measured alternatives that lost (tools/
// micro/fx_bench.hip): weights read from LDS just in time (~15 cycles a key
// of exposed latency), V prefetched through a four-slot register ring (the
// loop-carried wait counts came out vmcnt(0)) or an LDS-DMA ring (~60 cycles
// of issue per 1 KiB piece).
//
// keys [0, n) of one (head, sequence): the V^T rows of the wave's 64
// dimensions from vt (its key block 0, uniform), two register buffers in
// turn, the next step's loads issued before the current step's arithmetic --
// unconditionally (blocks past the sequence re-read its last one, fx_loadQ),
// so the wait counts stay exact.  c0: the first key of the current weights chunk.
// Two register buffers (one of lead): four measured slower at 64 x 30 s (the
// QKV + attention group 30.2 -> 32.4 us, 164 VGPRs) -- the batch chain does not
// wait on V^T latency.
__device__ __forceinline__ void fx_chain1(const uint16_t *__restrict__ vt, int loff, int c0, int n, int lastb, const float *w,
                                          unsigned long long flags, uint32_t kb, f16 &acc) {
    constexpr int NB = 2;
    u32x4 v[NB][DX_Q / 8];
#pragma unroll
    for (int i = 0; i < NB - 1; i++) fx_loadQ(v[i], vt, loff, c0 + i * DX_Q, lastb);
    for (int j0 = 0; j0 < n; j0 += NB * DX_Q) {
#pragma unroll
        for (int s = 0; s < NB; s++) {
            fx_loadQ(v[(s + NB - 1) % NB], vt, loff, c0 + j0 + (s + NB - 1) * DX_Q, lastb);
            fx_step1_m(v[s], j0 + s * DX_Q, n, w, flags, kb, acc);
        }
    }
}

// query head h of sequence b, wave wid (0, 1) running dimensions 64 wid +
// lane; the waves share nothing (each derives the weights itself).  sg: the
// row's scaled scores (global memory, or LDS in the one-launch kernel)
__device__ __forceinline__ void decode_attn_exact_body(const DecodeAttnArgs &a, const int h, const int b, const int wid,
                                                       const float *sg) {
    const int lane = threadIdx.x & 63;
    const int g = h / (a.n_head / a.n_kv_head);
    const int nkv = a.pos[b] + 1;
    const long vtc = vt_ctx(a.max_ctx);
    const int wu = __builtin_amdgcn_readfirstlane(wid);   // uniform: a scalar load base
    const uint16_t *vcol = a.vt + ((long)b * a.n_kv_head + g) * 128 * vtc + 64 * wu * 8;   // the wave's key block 0
    float M = -INFINITY, S = 0.0f;
    f16 acc = 0;
    for (int c0 = 0; c0 < nkv; c0 += DX_KC) {
        const int n = min(DX_KC, nkv - c0);
        float w[DX_B], wl;
        unsigned long long flags;
        const float Mold = M;
        const float *sc = sg + c0;
        uint32_t kb;
        const float Sc = fx_weights_reg([&](int j) { return sc[j]; }, n, M, w, flags, wl, &kb);
        S = (Mold == -INFINITY ? 0.0f : S * expf(Mold - M)) + Sc;
        fx_chain1(vcol, 8 * lane, c0, n, (nkv - 1) >> 3, w, flags, kb, acc);
    }
    const float ov = (float)acc * (S == 0.0f ? 0.0f : 1.0f / S);   // ggml: VKQ32 = fp32(VKQ16) * (1 / S)
    const long e = (long)b * a.n_head * 128 + h * 128 + 64 * wid + lane;
    if (a.outq) {   // Q8_0 for the o-proj of a decode batch: a 32-block = 32 lanes
        float am = fabsf(ov);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
        a.outq[e] = q8_quant(ov, am);
        if ((lane & 31) == 0) a.outd[e >> 5] = q8_scale(am);
    } else if (a.out32) {
        a.out32[e] = ov;
    } else {
        a.out[e] = f_to_u16(ov);
    }
}

}  // namespace qasr
