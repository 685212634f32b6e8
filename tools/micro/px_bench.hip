// px_bench.hip -- fa_exact.hip's exact prefill attention: the round-5 kernel
// (prefill_attn_exact_kernel) against the round-6 schedule
// (prefill_attn_exact2_kernel) on the same synthetic Q / K / V, bit for bit,
// with device time per launch.  Shapes: the utterance set's refill (128 x 405
// rows), configs[1]'s prompt (1 x 1211), a ragged batch with cached prefixes
// (seq_pos0), and the aligner's fp32-score form (1 x 2487).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize
//        -I../../include -I../../qwen3-asr.cpp_amd/csrc px_bench.hip -o px_bench
#include "../../qwen3-asr.cpp_amd/csrc/fa_exact.hip"
#include "px_v0.h"
#ifndef PX_ALT
#define PX_ALT 4   // the kernel compared with the round-5 one (px_v0.h): 3 = px_v3.h's, 4 = fa_exact.hip's (the product)
#endif
#if PX_ALT == 3
#include "px_v3.h"
#define PX_ALT_KERNEL prefill_attn_exact2_kernel
#else
#define PX_ALT_KERNEL prefill_attn_exact_kernel
#endif

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qasr;

static uint32_t rng_state = 12345u;
static float frand() {
    rng_state = rng_state * 1664525u + 1013904223u;
    return ((rng_state >> 9) * (1.0f / 8388608.0f)) - 0.5f;
}
static uint16_t h16(float f) { _Float16 h = (_Float16)f; return __builtin_bit_cast(uint16_t, h); }

struct Case {
    const char *name;
    std::vector<int> len, pos0;
    bool f32s;
    bool sink = false;   // key 0 of every sequence aligned with the queries (an attention sink: few new maxima)
};

static void run_case(const Case &cs, int reps) {
    const int NH = 16, NKV = 8, QD = NH * 128, KD = NKV * 128;
    const int B = (int)cs.len.size();
    int rows = 0, max_len = 0, max_ctx = 0;
    std::vector<int> row0(B), slot(B);
    for (int b = 0; b < B; b++) {
        row0[b] = rows;
        rows += cs.len[b];
        max_len = std::max(max_len, cs.len[b]);
        max_ctx = std::max(max_ctx, (cs.pos0.empty() ? 0 : cs.pos0[b]) + cs.len[b]);
        slot[b] = b;
    }
    max_ctx = (max_ctx + 63) / 64 * 64;
    const size_t kvn = (size_t)B * NKV * max_ctx * 128 + kKvPadRows * 128;
    std::vector<uint16_t> hq((size_t)rows * QD), hk(kvn), hv(kvn);
    for (auto &x : hq) x = h16(2.0f * frand());
    for (auto &x : hk) x = h16(2.0f * frand());
    for (auto &x : hv) x = h16(frand());
    if (cs.sink) {   // every query +4 in dimension 0, key 0 of each (sequence, kv head) 8 there: its score tops the row
        for (int r = 0; r < rows; r++)
            for (int hh = 0; hh < NH; hh++) hq[(size_t)r * QD + hh * 128] = h16(4.0f + frand());
        for (int b = 0; b < B; b++)
            for (int kh = 0; kh < NKV; kh++) hk[((size_t)b * NKV + kh) * max_ctx * 128] = h16(8.0f);
    }
    uint16_t *q, *k, *v, *o0, *o1;
    float *q32 = nullptr, *k32 = nullptr;
    int *meta;
    CK(hipMalloc(&q, hq.size() * 2)); CK(hipMalloc(&k, kvn * 2)); CK(hipMalloc(&v, kvn * 2));
    CK(hipMalloc(&o0, (size_t)rows * QD * 2)); CK(hipMalloc(&o1, (size_t)rows * QD * 2));
    CK(hipMemcpy(q, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(k, hk.data(), kvn * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(v, hv.data(), kvn * 2, hipMemcpyHostToDevice));
    CK(hipMemset(o0, 0, (size_t)rows * QD * 2)); CK(hipMemset(o1, 0xff, (size_t)rows * QD * 2));
    std::vector<int> hm;
    hm.insert(hm.end(), row0.begin(), row0.end());
    hm.insert(hm.end(), cs.len.begin(), cs.len.end());
    hm.insert(hm.end(), slot.begin(), slot.end());
    if (!cs.pos0.empty()) hm.insert(hm.end(), cs.pos0.begin(), cs.pos0.end());
    CK(hipMalloc(&meta, hm.size() * 4));
    CK(hipMemcpy(meta, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
    PrefillAttnArgs a{};
    a.q = q; a.kc = k; a.vc = v; a.seq_row0 = meta; a.seq_len = meta + B; a.seq_slot = meta + 2 * B;
    a.seq_pos0 = cs.pos0.empty() ? nullptr : meta + 3 * B;
    a.n_seq = B; a.max_len = max_len; a.n_head = NH; a.n_kv_head = NKV; a.max_ctx = max_ctx; a.scale = 1.0f / sqrtf(128.0f);
    if (cs.f32s) {
        std::vector<float> hq32((size_t)rows * QD), hk32((size_t)rows * KD);
        for (auto &x : hq32) x = 2.0f * frand();
        for (auto &x : hk32) x = 2.0f * frand();
        CK(hipMalloc(&q32, hq32.size() * 4)); CK(hipMalloc(&k32, hk32.size() * 4));
        CK(hipMemcpy(q32, hq32.data(), hq32.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(k32, hk32.data(), hk32.size() * 4, hipMemcpyHostToDevice));
        a.q32 = q32; a.k32 = k32;
    }
    dim3 grid((max_len + PX_ROWS - 1) / PX_ROWS, NH, B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best[2] = {1e30f, 1e30f};
    auto launch = [&](int ver) {
        PrefillAttnArgs av = a;
        av.out = ver ? o1 : o0;
        if (ver == 0) {
            if (cs.f32s) hipLaunchKernelGGL(prefill_attn_exact_r5_kernel<true>, grid, dim3(64 * PX_W), 0, 0, av);
            else hipLaunchKernelGGL(prefill_attn_exact_r5_kernel<false>, grid, dim3(64 * PX_W), 0, 0, av);
        } else {
            if (cs.f32s) hipLaunchKernelGGL(PX_ALT_KERNEL<true>, grid, dim3(64 * PX_W), 0, 0, av);
            else hipLaunchKernelGGL(PX_ALT_KERNEL<false>, grid, dim3(64 * PX_W), 0, 0, av);
        }
    };
    launch(0);
    launch(1);
    CK(hipDeviceSynchronize());
#ifdef FX_STAMPS
    {
        void *sp = nullptr;
        CK(hipGetSymbolAddress(&sp, HIP_SYMBOL(fx_stamps)));
        CK(hipMemset(sp, 0, (size_t)(1 << 16) * 8 * 8));
    }
#endif
    for (int r = 0; r < reps; r++) {   // alternating, best of reps each: clock / power drift hits both alike
        for (int ver = 0; ver < 2; ver++) {
            CK(hipEventRecord(e0, 0));
            launch(ver);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best[ver] = std::min(best[ver], ms);
        }
    }
#ifdef FX_STAMPS
    {   // v2 ran last: per-wave phase cycles (a sample of waves, fa_exact.hip PX_MARK)
        std::vector<unsigned long long> st((size_t)(1 << 16) * 8);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(fx_stamps), st.size() * 8));
        double ph[6] = {0, 0, 0, 0, 0, 0}, life = 0;
        long nw = 0;
        for (size_t e = 0; e < (size_t)(1 << 16); e++) {
            const unsigned long long *x = &st[e * 8];
            if (x[1] <= x[0]) continue;
            nw++;
            life += x[1] - x[0];
            for (int i = 0; i < 5; i++) ph[i] += x[2 + i];
            ph[5] += x[7];
        }
        if (nw) printf("    v2 phases (avg per wave, kcyc): life %.1f  barrier1 %.1f  scores %.1f  barrier2 %.1f  weights %.1f  chain %.1f  "
                       "pre-barrier %.1f  (%ld waves)\n", life / nw / 1e3, ph[0] / nw / 1e3, ph[1] / nw / 1e3, ph[2] / nw / 1e3,
                       ph[3] / nw / 1e3, ph[4] / nw / 1e3, ph[5] / nw / 1e3, nw);
    }
#endif
    std::vector<uint16_t> r0((size_t)rows * QD), r1((size_t)rows * QD);
    CK(hipMemcpy(r0.data(), o0, r0.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r1.data(), o1, r1.size() * 2, hipMemcpyDeviceToHost));
    size_t diff = 0, first = (size_t)-1;
    for (size_t i = 0; i < r0.size(); i++)
        if (r0[i] != r1[i]) {
            if (!diff) first = i;
            diff++;
        }
    if (diff) {   // the first differing element and how far off it is
        _Float16 a = __builtin_bit_cast(_Float16, r0[first]), b = __builtin_bit_cast(_Float16, r1[first]);
        long rr = (long)(first / QD);
        printf("    first diff: row %ld head %ld dim %ld: %04x (%g) vs %04x (%g)\n", rr, (long)(first % QD) / 128, (long)(first % 128),
               r0[first], (double)a, r1[first], (double)b);
        double maxrel = 0;
        for (size_t i = 0; i < r0.size(); i++) {
            const double x = (double)__builtin_bit_cast(_Float16, r0[i]), y = (double)__builtin_bit_cast(_Float16, r1[i]);
            maxrel = std::max(maxrel, std::fabs(x - y));
        }
        printf("    max |diff| %g\n", maxrel);
    }
    // chain VALU-issue bound: 3 wave-instructions per (row, key) pair of a head's two dimension
    // halves... = 3 per row-key per 64 lanes x 2 dims = per (row, head, key) 3 x 128 / 128 wave-instr
    double rk = 0;
    for (int b = 0; b < B; b++) {
        const int p0 = cs.pos0.empty() ? 0 : cs.pos0[b];
        for (int t = 0; t < cs.len[b]; t++) rk += p0 + t + 1;
    }
    const double instr = rk * NH * 3.0, bound_ms = instr * 4.0 / (1024.0 * 2.4e9) * 1e3;
    printf("%-28s rows %6d  v0 %8.1f us  v2 %8.1f us  (%.2fx)  chain bound %7.1f us -> v0 %.2f v2 %.2f  outputs differ: %zu of %zu\n",
           cs.name, rows, best[0] * 1e3, best[1] * 1e3, best[0] / best[1], bound_ms * 1e3, bound_ms / best[0], bound_ms / best[1],
           diff, r0.size());
    CK(hipFree(q)); CK(hipFree(k)); CK(hipFree(v)); CK(hipFree(o0)); CK(hipFree(o1)); CK(hipFree(meta));
    if (q32) { CK(hipFree(q32)); CK(hipFree(k32)); }
}

// px_expf_nonpos against the device expf on every x <= 0 (all 2^31 bit patterns with the sign set, and +0)
__global__ void expf_check(unsigned long long *bad) {
    const uint32_t base = (blockIdx.x * 256u + threadIdx.x) * 16u;
    unsigned long long nb = 0;
    for (uint32_t k = 0; k < 16; k++) {
        const uint32_t u = (base + k) | 0x80000000u;
        const float x = __uint_as_float(u);
        const float a = expf(x), b = px_expf_nonpos(x);
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) nb++;
    }
    if (base == 0) {
        const float a = expf(0.0f), b = px_expf_nonpos(0.0f);
        if (__float_as_uint(a) != __float_as_uint(b)) nb++;
    }
    if (nb) atomicAdd(bad, nb);
}

int main(int argc, char **argv) {
    {
        unsigned long long *bad, hb = 0;
        CK(hipMalloc(&bad, 8));
        CK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(expf_check, dim3(1u << 19), dim3(256), 0, 0, bad);
        CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("px_expf_nonpos vs expf over all 2^31 x <= 0: %llu differ\n", hb);
        CK(hipFree(bad));
    }
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    std::vector<Case> cases;
    cases.push_back({"batch 128 x 405", std::vector<int>(128, 405), {}, false});
    cases.push_back({"configs[1] 1 x 1211", {1211}, {}, false});
    cases.push_back({"batch 128 x 405, key-0 sink", std::vector<int>(128, 405), {}, false, true});
    {
        Case c{"ragged 24, cached prefixes", {}, {}, false};
        for (int b = 0; b < 24; b++) { c.len.push_back(17 + 37 * b % 400); c.pos0.push_back((b % 3) * 61); }
        cases.push_back(c);
    }
    cases.push_back({"aligner fp32 1 x 2487", {2487}, {}, true});
    cases.push_back({"aligner fp32 batch 8 x 700", std::vector<int>(8, 700), {}, true});
    const int only = argc > 2 ? atoi(argv[2]) : -1;   // one case (profiling passes)
    for (int i = 0; i < (int)cases.size(); i++)
        if (only < 0 || only == i) run_case(cases[i], reps);
    return 0;
}
