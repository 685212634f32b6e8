// ffn_roles.h -- the batch-1 FFN's two workgroup roles (text_decoder.cpp:
// 545-560: rms_norm * w -> silu(gate) * up -> down + residual), shared by
// gemv.hip's ffn1_kernel: one wave per OPW outputs, the
// gemv1_kernel lane split and wave_sum order (bit-identical to gemv1_kernel).
//
// Gate/up role: OPW SwiGLU outputs per wave (16-row interleave: output o =
// weight rows 32 (o / 16) + o % 16 and + 16), x RMS-normalised per wave; the
// block's 4 OPW fp16 outputs leave as write-through 32-bit stores, the wave
// drains, and lane 0 counts the block into shard blk % 32 of the layer's
// arrival counter (MI355X_MICROARCH.md inter-workgroup hand-off: 32 shards
// instead of one counter that serialises every arrival at the memory side).
//
// Down role: RPW rows per wave (+ residual); weights requested after wdelay,
// then one wave polls the gate/up shards and the activation is read with sc1
// loads.
#pragma once
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

__device__ __forceinline__ float silu1(float g) { return g / (1.0f + expf(-g)); }


// six 16-B sc1 loads: 3072 fp16 activations of lane `p` (lane * 8 + t * 512)
__device__ __forceinline__ void ld_sc1_x4_6(const uint16_t *p, u32x4 *v) {
    asm volatile(
        "global_load_dwordx4 %0, %6, off sc1\n\t"
        "global_load_dwordx4 %1, %6, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %6, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %6, off offset:3072 sc1\n\t"
        "global_load_dwordx4 %4, %7, off sc1\n\t"
        "global_load_dwordx4 %5, %7, off offset:1024 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5])
        : "v"(p), "v"(p + 2048)
        : "memory");
}
// one wave polls 32 shards (lane s: shard s) until each holds `need`; bounded
// by poll_limit, a wait that runs out sets errbit; the verdict in *ready
__device__ __forceinline__ void ffn_wait_shards(const unsigned int *cnt, unsigned need, int delay, int poll_limit, int fence,
                                                unsigned int *err, unsigned errbit, int *ready) {
    const int lane = threadIdx.x & 63;
    for (int i = 0; i < delay; i++) __builtin_amdgcn_s_sleep(8);
    int ok = 0;
    for (int it = 0; it < poll_limit; it++) {
        const unsigned v = lane < 32 ? __hip_atomic_load(cnt + lane * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
        if (__all(v >= need)) { ok = 1; break; }
        __builtin_amdgcn_s_sleep(8);
    }
    if (fence) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (lane == 0) {
        *ready = ok;
        if (!ok) __hip_atomic_fetch_or(err, errbit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// gate/up role, block blk of the role (4 waves x OPW outputs)
template <int K, int OPW>
__device__ __forceinline__ void ffn_gu_role(const GemvArgs &g, const GemvArgs &d, const FfnCtl &c, int blk) {
    constexpr int NT = K / 512;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (g.trace && threadIdx.x == 0) g.trace[blk * 8] = rt_now();
    if (blk == 0 && threadIdx.x < 32) {   // re-arm the next layer's shards (their last use ended a step ago)
        c.cnt_next[threadIdx.x * 16] = 0u;
        if (d.zero8 && threadIdx.x < 8) d.zero8[threadIdx.x * 16] = 0u;   // the fused o-proj's counters
    }
    half8 wv[OPW][2][NT];
#pragma unroll
    for (int i = 0; i < OPW; i++) {
        const int o = (blk * 4 + wid) * OPW + i;
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int t = 0; t < NT; t++)
                wv[i][q][t] = __builtin_nontemporal_load((const half8 *)(g.W + (32L * (o >> 4) + (o & 15) + 16 * q) * K + t * 512 + lane * 8));
    }
    float xf[NT][8];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const float4 a = *(const float4 *)(g.x + t * 512 + lane * 8);
        const float4 b = *(const float4 *)(g.x + t * 512 + lane * 8 + 4);
        xf[t][0] = a.x; xf[t][1] = a.y; xf[t][2] = a.z; xf[t][3] = a.w;
        xf[t][4] = b.x; xf[t][5] = b.y; xf[t][6] = b.z; xf[t][7] = b.w;
    }
    double ss = 0.0;   // ggml_rms_norm: double sum of fp32 squares
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int e = 0; e < 8; e++) ss += (double)(xf[t][e] * xf[t][e]);
    ss = wave_sum_d(ss);
    const float scale = 1.0f / sqrtf((float)(ss / K) + g.eps);
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const float4 a = *(const float4 *)(g.norm_w + t * 512 + lane * 8);
        const float4 b = *(const float4 *)(g.norm_w + t * 512 + lane * 8 + 4);
        const float w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; e++) xf[t][e] = (float)f2h(fmul_rn(fmul_rn(xf[t][e], scale), w[e]));
    }
    __shared__ uint16_t outs[4 * OPW];
#pragma unroll
    for (int i = 0; i < OPW; i++) {
        float acc[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            acc[q] = 0.f;
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int e = 0; e < 8; e++) acc[q] = fmaf((float)wv[i][q][t][e], xf[t][e], acc[q]);
            acc[q] = wave_sum(acc[q]);
        }
        if (lane == 0) outs[wid * OPW + i] = f_to_u16(silu1(acc[0]) * acc[1]);
    }
    __syncthreads();
    if (wid == 0) {
        if (lane < 2 * OPW)
            __hip_atomic_store((uint32_t *)(g.out_f16 + blk * 4 * OPW) + lane, (uint32_t)outs[2 * lane] | ((uint32_t)outs[2 * lane + 1] << 16),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (c.fence) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) __hip_atomic_fetch_add(c.cnt + (blk & 31) * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (g.trace && threadIdx.x == 0) g.trace[blk * 8 + 1] = rt_now();
}

// down role, block j of the role (4 waves x RPW rows); need = gate/up blocks / 32
template <int F, int RPW>
__device__ __forceinline__ void ffn_dn_role(const GemvArgs &d, const FfnCtl &c, int j, unsigned need) {
    constexpr int NTD = F / 512;
    static_assert(NTD == 6, "ld_sc1_x4_6 covers F = 3072");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (d.trace && threadIdx.x == 0) d.trace[j * 8] = rt_now();
    for (int i = 0; i < c.wdelay; i++) __builtin_amdgcn_s_sleep(8);   // let the gate/up stream go first
    half8 wv[RPW][NTD];
#pragma unroll
    for (int r = 0; r < RPW; r++) {
        const int row = (j * 4 + wid) * RPW + r;
#pragma unroll
        for (int t = 0; t < NTD; t++) wv[r][t] = __builtin_nontemporal_load((const half8 *)(d.W + (long)row * F + t * 512 + lane * 8));
    }
    // one polling lane per shard, and only once the gate/up stream is nearly
    // done: pollers beside a weight stream cost it bandwidth (MI355X_MICROARCH.md, polling-cost)
    __shared__ int ready;
    if (wid == 0) ffn_wait_shards(c.cnt, need, c.delay, c.poll_limit, c.fence, c.err, DEVERR_FFN_WAIT, &ready);
    __syncthreads();
    if (!ready) return;   // reported through the error word; x keeps its old row
    u32x4 xv[NTD];
    ld_sc1_x4_6(d.xh + lane * 8, xv);
#pragma unroll
    for (int r = 0; r < RPW; r++) {
        const int row = (j * 4 + wid) * RPW + r;
        const float res = d.res[row];
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < NTD; t++) {
            const half8 h = __builtin_bit_cast(half8, xv[t]);
#pragma unroll
            for (int e = 0; e < 8; e++) acc = fmaf((float)wv[r][t][e], (float)h[e], acc);
        }
        acc = wave_sum(acc);
        if (lane == 0) d.out_f32[row] = fadd_rn(acc, res);
    }
    if (d.trace && threadIdx.x == 0) d.trace[j * 8 + 1] = rt_now();
}

}  // namespace qasr
