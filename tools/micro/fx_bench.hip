// Stand-alone timing of the round-5 exact prefill kernel (px_v0.h) at configs[1]'s shape
// (one 1211-row prompt, 16 heads, GQA 2:1, hd 128) with per-workgroup phase
// stamps (FX_STAMPS).  Build: see tools/micro/Makefile.
#define FX_STAMPS 1
#include "../../qwen3-asr.cpp_amd/csrc/fa_exact.hip"
#include "px_v0.h"   // the round-5 prefill kernel, the one with the phase stamps
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
using namespace qasr;

// the decode chain alone, one wave: (a) fx_chain1 as the kernel runs it, (b) the
// same batch arithmetic on register data only
__global__ void chain_only(const uint16_t *vt, int n, unsigned long long *cyc, uint16_t *out, int mode) {
    float w[DX_B], m[DX_B];
    for (int i = 0; i < DX_B; i++) { w[i] = 0.001f * (i & 7) + threadIdx.x * 1e-5f; m[i] = 1.0f; }
    f16 acc = 0;
    const unsigned long long t0 = clock64();
    if (mode == 0) {
        fx_chain1(vt, threadIdx.x * 8, 0, n, 1 << 28, w, 0ull, 0u, acc);   // every key on the fast path
    } else {
        u32x4 v[DX_B / 8];
        for (int i = 0; i < DX_B / 8; i++) v[i] = ((const u32x4 *)vt)[threadIdx.x * 200 + i];
        for (int j = 0; j < n; j += DX_B)
#pragma unroll
            for (int i = 0; i < DX_B; i++) acc = fx_mad1(acc, fx_elem(v, i), fx_lane(w[i], 3));
    }
    const unsigned long long t1 = clock64();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    out[threadIdx.x] = __builtin_bit_cast(uint16_t, acc);
}

int main(int argc, char **argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 1211, NH = 16, NKV = 8, CTX = L + 64;
    std::vector<uint16_t> hq((size_t)L * NH * 128), hk((size_t)NKV * CTX * 128 + kKvPadRows * 128), hv(hk.size());
    srand(1);
    auto rh = [](float s) { _Float16 h = (_Float16)(s * ((rand() & 0xffff) / 32768.0f - 1.0f)); return __builtin_bit_cast(uint16_t, h); };
    for (auto &x : hq) x = rh(1.0f);
    for (auto &x : hk) x = rh(1.0f);
    for (auto &x : hv) x = rh(0.5f);
    uint16_t *q, *k, *v, *o;
    int *meta;
    hipMalloc(&q, hq.size() * 2); hipMalloc(&k, hk.size() * 2); hipMalloc(&v, hv.size() * 2);
    hipMalloc(&o, hq.size() * 2); hipMalloc(&meta, 16);
    hipMemcpy(q, hq.data(), hq.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(k, hk.data(), hk.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(v, hv.data(), hv.size() * 2, hipMemcpyHostToDevice);
    int hm[4] = {0, L, 0, 0};   // row0, len, slot
    hipMemcpy(meta, hm, 16, hipMemcpyHostToDevice);
    PrefillAttnArgs a{};
    a.q = q; a.kc = k; a.vc = v; a.seq_row0 = meta; a.seq_len = meta + 1; a.seq_slot = meta + 2; a.n_seq = 1; a.max_len = L;
    a.n_head = NH; a.n_kv_head = NKV; a.max_ctx = CTX; a.scale = 1.0f / sqrtf(128.0f); a.out = o;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto launch_r5 = [&]() {
        hipLaunchKernelGGL(prefill_attn_exact_r5_kernel<false>, dim3((L + PX_ROWS - 1) / PX_ROWS, NH, 1), dim3(64 * PX_W), 0, 0, a);
    };
    for (int i = 0; i < 3; i++) launch_r5();
    hipEventRecord(e0, 0);
    const int reps = 10;
    for (int i = 0; i < reps; i++) launch_r5();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("prefill_attn_exact_r5_kernel L=%d: %.1f us per launch\n", L, ms * 1e3 / reps);
    const int nb = (L + 15) / 16 * NH;
    std::vector<unsigned long long> st((size_t)nb * 8);
    hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(fx_stamps), st.size() * 8);
    unsigned long long t0 = ~0ull, t1 = 0;
    double life = 0, ph[3] = {0, 0, 0}, ch = 0;
    for (int b = 0; b < nb; b++) {
        const unsigned long long *s = &st[(size_t)b * 8];
        t0 = std::min(t0, s[0]); t1 = std::max(t1, s[1]);
        life += s[1] - s[0];
        for (int i = 0; i < 3; i++) ph[i] += s[2 + i];
        ch += s[5];
    }
    printf("blocks %d  span %.0f kcyc  avg life %.1f kcyc  per block: scores %.1f  weights %.1f  chain %.1f kcyc  chunks %.1f\n",
           nb, (t1 - t0) / 1e3, life / nb / 1e3, ph[0] / nb / 1e3, ph[1] / nb / 1e3, ph[2] / nb / 1e3, ch / nb);
    // the longest block (q0 max, head 0)
    const unsigned long long *s = &st[0];
    printf("longest block q0=%llu: life %.1f  scores %.1f  weights %.1f  chain %.1f kcyc, chunks %llu\n", s[6], (s[1] - s[0]) / 1e3,
           s[2] / 1e3, s[3] / 1e3, s[4] / 1e3, s[5]);
    // decode chain at batch 1: context L + 49 keys (configs[1]'s first decode steps)
    {
        const int nkv = L + 49, vtc = vt_ctx(CTX);
        std::vector<float> hs((size_t)NH * CTX + 4096);
        for (auto &x : hs) x = 2.0f * ((rand() & 0xffff) / 32768.0f - 1.0f);
        std::vector<uint16_t> ht((size_t)NKV * 128 * vtc);
        for (auto &x : ht) x = rh(0.5f);
        float *sc; uint16_t *vt, *ao; int *pos;
        hipMalloc(&sc, hs.size() * 4); hipMalloc(&vt, ht.size() * 2); hipMalloc(&ao, NH * 128 * 2); hipMalloc(&pos, 4);
        hipMemcpy(sc, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(vt, ht.data(), ht.size() * 2, hipMemcpyHostToDevice);
        const int p = nkv - 1;
        hipMemcpy(pos, &p, 4, hipMemcpyHostToDevice);
        DecodeAttnArgs d{};
        d.scores = sc; d.vt = vt; d.pos = pos; d.B = 1; d.n_head = NH; d.n_kv_head = NKV; d.max_ctx = CTX; d.out = ao;
        for (int i = 0; i < 3; i++) launch_decode_attention_exact(d, 0);
        hipEventRecord(e0, 0);
        for (int i = 0; i < 20; i++) launch_decode_attention_exact(d, 0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("decode_attn_exact_kernel B=1 n_kv=%d: %.2f us per launch (incl. launch gaps)\n", nkv, ms * 1e3 / 20);
        {   // CPU restatement of ggml's loop on the same scores / V: max |diff| of the outputs
            std::vector<uint16_t> go(NH * 128);
            hipMemcpy(go.data(), ao, NH * 128 * 2, hipMemcpyDeviceToHost);
            double worst = 0;
            for (int hh = 0; hh < NH; hh++) {
                const int g = hh / (NH / NKV);
                std::vector<_Float16> acc(128, (_Float16)0.0f);
                float M = -INFINITY, S = 0;
                for (int k = 0; k < nkv; k++) {
                    const float sv = hs[(size_t)hh * CTX + k];
                    float ms = 1, vsw = 1;
                    if (sv > M) { const float Mo = M; M = sv; ms = expf(Mo - M);
                        for (int d = 0; d < 128; d++) acc[d] = (_Float16)((float)acc[d] * ms);
                    } else vsw = expf(sv - M);
                    for (int d = 0; d < 128; d++) {
                        const uint16_t u = ht[(size_t)g * 128 * vtc + vt_index(k, d)];
                        acc[d] = (_Float16)fmaf((float)__builtin_bit_cast(_Float16, u), vsw, (float)acc[d]);
                    }
                    S = S * ms + vsw;
                }
                for (int d = 0; d < 128; d++) {
                    const float ref = (float)acc[d] / S;
                    const float got = (float)__builtin_bit_cast(_Float16, go[hh * 128 + d]);
                    worst = std::max(worst, (double)fabsf(ref - got));
                }
            }
            printf("  vs CPU ggml loop: max |diff| %.3g\n", worst);
        }
        std::vector<unsigned long long> ds(32 * 8);
        hipMemcpyFromSymbol(ds.data(), HIP_SYMBOL(fx_stamps), ds.size() * 8, 60000 * 8 * 8);
        for (int w = 0; w < 4; w++)
            printf("  wave %d: life %.1f kcyc  weights %.1f  chain %.1f\n", w, (ds[w * 8 + 1] - ds[w * 8]) / 1e3, ds[w * 8 + 2] / 1e3,
                   ds[w * 8 + 3] / 1e3);
        d.B = 64;
        std::vector<int> p64(64, p);
        int *pos64; float *sc64; uint16_t *vt64, *ao64;
        hipMalloc(&pos64, 256); hipMalloc(&sc64, hs.size() * 4 * 64); hipMalloc(&vt64, ht.size() * 2 * 64); hipMalloc(&ao64, 64 * NH * 128 * 2);
        hipMemset(sc64, 0, hs.size() * 4 * 64); hipMemset(vt64, 0, ht.size() * 2 * 64);
        hipMemcpy(pos64, p64.data(), 256, hipMemcpyHostToDevice);
        d.pos = pos64; d.scores = sc64; d.vt = vt64; d.out = ao64;
        launch_decode_attention_exact(d, 0);
        hipEventRecord(e0, 0);
        for (int i = 0; i < 10; i++) launch_decode_attention_exact(d, 0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("decode_attn_exact_kernel B=64 n_kv=%d: %.2f us per launch\n", nkv, ms * 1e3 / 10);
    }
    {
        uint16_t *vt; unsigned long long *cyc; uint16_t *out;
        hipMalloc(&vt, 1800 * 128 * 2 + 4096); hipMalloc(&cyc, 8); hipMalloc(&out, 128);
        hipMemset(vt, 0, 1800 * 128 * 2 + 4096);
        for (int mode = 0; mode < 2; mode++) {
            unsigned long long c = 0;
            for (int r = 0; r < 3; r++) {
                hipLaunchKernelGGL(chain_only, dim3(1), dim3(64), 0, 0, vt, 1280, cyc, out, mode);
                hipDeviceSynchronize();
            }
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("chain_only mode %d (%s): %.2f cycles/key\n", mode, mode ? "registers" : "fx_chain1", c / 1280.0);
        }
    }
    return 0;
}
