// q8_gemm_bench.hip -- the Q8_0 block GEMM of the encoder / prefill projections
// (csrc/gemm_q8.hip, included directly): us per launch of the engine's
// register-staged tile against an LDS-DMA ring form of the same tile (defined
// here; measured no faster at any (KS, NB)) and against the same
// products on the fp16 MFMA (int8 quants held as fp16 values: exact; also
// defined here, also slower), each output compared bit for bit with the engine
// tile's.  The fp16 form reads GemmArgs::A / W as the fp16 quants and its own
// wd32 argument as the fp32 W scales.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form=1
#include "../../qwen3-asr.cpp_amd/csrc/gemm_q8.hip"

namespace qasr {
// ------------------------------------------------- Q8_0 GEMM, LDS-DMA ring
// The same tile, fragments, per-block arithmetic and epilogue as gemm_q8_kernel
// (so the same bits), with every operand moved global -> LDS by LDS-DMA through
// an NB-deep ring of stages (gemm_glds_kernel's scheme): no staging registers,
// no ds_write pass, NB - 1 stages in flight behind the one being multiplied.
// A stage is KS 32-wide K blocks:
//   quants: 1-KiB pieces of whole stage rows (KS * 32 B: A rows, then W rows);
//     lane l lands at row l / CPR, 16-B position l % CPR and fetches chunk
//     (l % CPR) ^ ((row >> SWS) & (CPR - 1)), so the 16 rows of an 8-byte
//     fragment read fall in distinct bank groups (an earlier form with 32-B
//     rows per block, two lanes a row, ran 3-10 % slower still);
//   per block, A scales: fp32, one dword a lane (row m0 + 64h + l), stored per block as a
//     row vector (the C layout's 4 consecutive rows are one ds_read_b128);
//   W scales: the fp16 pair of blocks (2v, 2v + 1) of row n0 + l, one dword a lane.
// Rows past M fetch a global zero line; the per-wave piece count is made
// uniform with dummy pieces into a scratch KiB (vmcnt counts them).
typedef __attribute__((address_space(3))) void lds_void_q;
typedef __attribute__((address_space(1))) void glb_void_q;
__device__ __attribute__((aligned(64))) uint32_t g_zero_line_q[16];

template <int N>
__device__ __forceinline__ void wait_vm_q() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int KS, int NB, int EPI>
__global__ __launch_bounds__(256) void gemm_q8_glds_kernel(GemmArgs g) {
    constexpr int FM = BM / 32, FN = BN / 32;
    constexpr int ROWS = BM + BN;
    static_assert(BM == 128 && BN == 64 && (KS == 2 || KS == 4) && NB >= 2 && NB <= 4, "tile");
    constexpr int RB = KS * 32;                   // quant bytes per row per stage
    constexpr int CPR = RB / 16;                  // 16-B chunks per row
    constexpr int RPP = 64 / CPR;                 // rows per 1-KiB piece
    constexpr int SWS = KS == 2 ? 2 : 1;          // swizzle: chunk ^ ((row >> SWS) & (CPR - 1))
    constexpr int QB = ROWS * RB;                 // quant bytes per stage
    constexpr int QP = ROWS / RPP;                // quant pieces per stage
    constexpr int AP = BM / 64;                   // A-scale pieces per block
    constexpr int NP = QP + KS * AP + KS / 2;     // pieces per stage
    constexpr int NW = (NP + 3) / 4;              // per wave (uniform)
    constexpr int STG = QB + KS * BM * 4 + (KS / 2) * BN * 4;   // bytes per stage
    static_assert((NB - 2) * NW < 64, "vmcnt range");
    __shared__ __attribute__((aligned(16))) uint8_t smem[NB * STG + 1024];
    uint8_t *scratch = smem + NB * STG;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int M = g.M, K = g.K, nbw = K / 32;

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int kb0, int buf) {   // kb0: the stage's first K block
        uint8_t *st = smem + buf * STG;
#pragma unroll
        for (int p = 0; p < NW; p++) {
            const int i = wid + 4 * p;   // wave-uniform
            if (i < QP) {
                const int r = i * RPP + lane / CPR;
                const int ch = (lane % CPR) ^ ((r >> SWS) & (CPR - 1));
                const int8_t *src = (const int8_t *)g_zero_line_q;
                if (r < BM) {
                    if (m0 + r < M) src = g.Aq + (long)(m0 + r) * g.lda + kb0 * 32 + ch * 16;
                } else {
                    src = g.Wq + (long)(n0 + r - BM) * g.ldw + kb0 * 32 + ch * 16;
                }
                __builtin_amdgcn_global_load_lds((glb_void_q *)src, (lds_void_q *)(st + i * 1024), 16, 0, 0);
            } else if (i < QP + KS * AP) {
                const int j = i - QP, u = j / AP, h = j - u * AP;
                const int row = m0 + h * 64 + lane;
                const float *src = row < M ? g.Ad + (long)row * g.ldad + kb0 + u : (const float *)g_zero_line_q;
                __builtin_amdgcn_global_load_lds((glb_void_q *)src, (lds_void_q *)(st + QB + (u * BM + h * 64) * 4), 4, 0, 0);
            } else if (i < NP) {
                const int v = i - QP - KS * AP;
                const uint16_t *src = g.Wd + (long)(n0 + lane) * nbw + kb0 + 2 * v;
                __builtin_amdgcn_global_load_lds((glb_void_q *)src, (lds_void_q *)(st + QB + KS * BM * 4 + v * BN * 4), 4, 0, 0);
            } else {
                __builtin_amdgcn_global_load_lds((glb_void_q *)g_zero_line_q, (lds_void_q *)scratch, 16, 0, 0);
            }
        }
    };

    const int nk = K / (32 * KS);
#pragma unroll
    for (int st = 0; st < NB - 1; st++)
        if (st < nk) issue(st * KS, st);
    const int kg = lane >> 4;
    int buf = 0;
    for (int kt = 0; kt < nk; kt++) {
        const int ahead = nk - 1 - kt;
        if constexpr (NB >= 4) {
            if (ahead >= 2) wait_vm_q<2 * NW>();
            else if (ahead == 1) wait_vm_q<NW>();
            else wait_vm_q<0>();
        } else if constexpr (NB == 3) {
            if (ahead >= 1) wait_vm_q<NW>();
            else wait_vm_q<0>();
        } else {
            wait_vm_q<0>();
        }
        asm volatile("s_barrier" ::: "memory");   // every wave's pieces landed; stage kt-1's readers done
        if (kt + NB - 1 < nk) {
            int nb = buf + NB - 1;
            if (nb >= NB) nb -= NB;
            issue((kt + NB - 1) * KS, nb);
        }
        const uint8_t *st = smem + buf * STG;
#pragma unroll 1
        for (int u = 0; u < KS; u++) {
            const float *asc = (const float *)(st + QB) + u * BM;
            const uint32_t *wsc = (const uint32_t *)(st + QB + KS * BM * 4) + (u >> 1) * BN;
            const int gch = 2 * u + (kg >> 1), inner = (kg & 1) << 3;   // the fragment's chunk in the row
            long af[FM], bf[FN];
            floatx4 sa[FM];
            float sb[FN];
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const int r = wr * (BM / 2) + i * 16 + (lane & 15);
                af[i] = *(const long *)(st + r * RB + (((gch ^ ((r >> SWS) & (CPR - 1))) << 4) | inner));
                sa[i] = *(const floatx4 *)(asc + wr * (BM / 2) + i * 16 + 4 * kg);
            }
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int r = BM + wc * (BN / 2) + j * 16 + (lane & 15);
                bf[j] = *(const long *)(st + r * RB + (((gch ^ ((r >> SWS) & (CPR - 1))) << 4) | inner));
                const uint32_t h = wsc[r - BM];
                sb[j] = u16_to_f((uint16_t)((u & 1) ? h >> 16 : h & 0xffffu));
            }
            // gemm_q8_kernel's pinned order: fragment f's MFMA, then f - 1's scaling
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
        if (++buf == NB) buf = 0;
    }
    gemm_epilogue<BM, BN, EPI>(g, acc, m0, n0, wr, wc, lane);
}

template <int BM, int BN, int KS, int NB, int EPI>
static void run_gemm_q8_glds(const GemmArgs &g, hipStream_t s) {
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    hipLaunchKernelGGL((gemm_q8_glds_kernel<BM, BN, KS, NB, EPI>), grid, dim3(256), 0, s, g);
}


// ---------------------------------------- Q8_0 GEMM on the fp16 MFMA, LDS-DMA
// gemm_glds_kernel's ring, pieces, swizzle and epilogue (gemm.hip) over fp16
// operands that hold int8 quants, one 32-deep slab a Q8_0 block: per slab and
// fragment one v_mfma_f32_16x16x32_f16 from a zero accumulator -- exact, the
// (float)sumi of v_mfma_i32_16x16x32_i8 + v_cvt -- scaled into the fp32
// accumulator as gemm_q8_kernel does (q8_scale_acc's packed mul + fma), so the
// same bits, with 4 VALU a MFMA instead of 8 and the f16 tile's staging.  The
// block scales ride the ring as dword LDS-DMA pieces (64 rows each, fp32 row
// vectors per slab: the C layout's 4 consecutive A rows are one ds_read_b128).
typedef __attribute__((address_space(3))) void lds_void_h;
typedef __attribute__((address_space(1))) void glb_void_h;
__device__ __attribute__((aligned(64))) uint32_t g_zero_line_h[16];

template <int N>
__device__ __forceinline__ void wait_vm_h() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int KS, int NB, int EPI, int WNW>
__global__ __launch_bounds__(128 * WNW) void gemm_q8h_kernel(GemmArgs g, const float *wd32) {
    constexpr int NWAVE = 2 * WNW;
    constexpr int FM = BM / 32, FN = BN / (16 * WNW);
    constexpr int ROWS = BM + BN;
    constexpr int SLAB = ROWS * 32;                  // halves per 32-deep slab
    constexpr int RG = ROWS / 16;                    // 1-KiB quant pieces per slab
    constexpr int SP = ROWS / 64;                    // scale pieces per slab (A rows, then W rows)
    constexpr int NP = KS * (RG + SP);               // pieces per stage
    constexpr int NW = (NP + NWAVE - 1) / NWAVE;     // per wave (uniform: vmcnt counts)
    constexpr int STG = KS * SLAB * 2 + KS * ROWS * 4;   // bytes per stage
    static_assert(BM % 64 == 0 && BN % 64 == 0 && NB >= 2 && NB <= 4 && (NB - 2) * NW < 64, "tile");
    __shared__ __attribute__((aligned(16))) uint8_t smem[NB * STG + 1024];
    uint8_t *scratch = smem + NB * STG;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid / WNW, wc = wid % WNW;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int M = g.M, K = g.K, nbw = K / 32;
    const uint16_t *A = g.A, *W = g.W;

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int lrow = lane >> 2, lpos = lane & 3;
    auto issue = [&](int kb0, int buf) {   // kb0: the stage's first 32-block
        uint8_t *st = smem + buf * STG;
#pragma unroll
        for (int p = 0; p < NW; p++) {
            const int i = wid + NWAVE * p;   // wave-uniform
            if (i < KS * RG) {
                const int s = i / RG, rg = i - s * RG;
                const int r = rg * 16 + lrow;
                const int k = (kb0 + s) * 32 + ((lpos ^ ((r >> 1) & 3)) << 3);
                const uint16_t *src = (const uint16_t *)g_zero_line_h;
                if (rg * 16 < BM) {
                    if (m0 + r < M) src = A + (long)(m0 + r) * g.lda + k;
                } else {
                    src = W + (long)(n0 + r - BM) * g.ldw + k;
                }
                __builtin_amdgcn_global_load_lds((glb_void_h *)src, (lds_void_h *)(st + (s * SLAB + rg * 512) * 2), 16, 0, 0);
            } else if (i < NP) {
                const int j = i - KS * RG, s = j / SP, h = j - s * SP;
                const int r = h * 64 + lane;   // scale row of the slab: A rows, then W rows
                const float *src = (const float *)g_zero_line_h;
                if (r < BM) {
                    if (m0 + r < M) src = g.Ad + (long)(m0 + r) * g.ldad + kb0 + s;
                } else {
                    src = wd32 + (long)(n0 + r - BM) * nbw + kb0 + s;
                }
                __builtin_amdgcn_global_load_lds((glb_void_h *)src, (lds_void_h *)(st + KS * SLAB * 2 + (s * ROWS + h * 64) * 4), 4, 0, 0);
            } else {
                __builtin_amdgcn_global_load_lds((glb_void_h *)g_zero_line_h, (lds_void_h *)scratch, 16, 0, 0);
            }
        }
    };

    const int nk = K / (32 * KS);
#pragma unroll
    for (int st = 0; st < NB - 1; st++)
        if (st < nk) issue(st * KS, st);
    const int q = lane >> 4;
    int buf = 0;
    for (int kt = 0; kt < nk; kt++) {
        const int ahead = nk - 1 - kt;
        if constexpr (NB >= 4) {
            if (ahead >= 2) wait_vm_h<2 * NW>();
            else if (ahead == 1) wait_vm_h<NW>();
            else wait_vm_h<0>();
        } else if constexpr (NB == 3) {
            if (ahead >= 1) wait_vm_h<NW>();
            else wait_vm_h<0>();
        } else {
            wait_vm_h<0>();
        }
        asm volatile("s_barrier" ::: "memory");   // every wave's pieces landed; stage kt-1's readers done
        if (kt + NB - 1 < nk) {
            int nb = buf + NB - 1;
            if (nb >= NB) nb -= NB;
            issue((kt + NB - 1) * KS, nb);
        }
        const uint8_t *st = smem + buf * STG;
#pragma unroll
        for (int s = 0; s < KS; s++) {
            const uint16_t *sl = (const uint16_t *)st + s * SLAB;
            const float *sc = (const float *)(st + KS * SLAB * 2) + s * ROWS;
            half8 af[FM], bf[FN];
            floatx4 sa[FM];
            float sb[FN];
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const int r = wr * (BM / 2) + i * 16 + (lane & 15);
                af[i] = *(const half8 *)(sl + r * 32 + ((q ^ ((r >> 1) & 3)) << 3));
                sa[i] = *(const floatx4 *)(sc + wr * (BM / 2) + i * 16 + 4 * q);
            }
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int r = BM + wc * (BN / WNW) + j * 16 + (lane & 15);
                bf[j] = *(const half8 *)(sl + r * 32 + ((q ^ ((r >> 1) & 3)) << 3));
                sb[j] = sc[r];
            }
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int j = 0; j < FN; j++) {
                    const floatx4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                    const floatx2 w2 = {sb[j], sb[j]};
                    const floatx2 s01 = w2 * floatx2{sa[i][0], sa[i][1]}, s23 = w2 * floatx2{sa[i][2], sa[i][3]};
                    const floatx2 a01 = __builtin_elementwise_fma(s01, floatx2{c[0], c[1]}, floatx2{acc[i][j][0], acc[i][j][1]});
                    const floatx2 a23 = __builtin_elementwise_fma(s23, floatx2{c[2], c[3]}, floatx2{acc[i][j][2], acc[i][j][3]});
                    acc[i][j] = floatx4{a01[0], a01[1], a23[0], a23[1]};
                }
        }
        if (++buf == NB) buf = 0;
    }
    gemm_epilogue<BM, BN, EPI, WNW>(g, acc, m0, n0, wr, wc, lane);
}

template <int BM, int BN, int KS, int NB, int EPI, int WNW>
static void run_gemm_q8h(const GemmArgs &g, const float *wd32, hipStream_t s) {
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    hipLaunchKernelGGL((gemm_q8h_kernel<BM, BN, KS, NB, EPI, WNW>), grid, dim3(128 * WNW), 0, s, g, wd32);
}

}  // namespace qasr

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace qasr;

template <typename F>
static double timeit(F launch, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    launch();
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(a, s));
        for (int r = 0; r < 5; r++) launch();
        CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    return best * 1e3 / 5;
}

int main() {
    hipStream_t s; CK(hipStreamCreate(&s));
    struct Sh { const char *name; int M, N, K; };
    const Sh shapes[] = {{"enc qkv b64", 24960, 2688, 896}, {"enc fc1 b64", 24960, 3584, 896}, {"enc fc2 b64", 24960, 896, 3584},
                         {"prefill qkv b64", 25920, 4096, 1024}, {"prefill down b64", 25920, 1024, 3072}, {"odd M", 2500, 1024, 1024}};
    const size_t MA = (size_t)25920 * 3584, MW = (size_t)4096 * 3584, MO = (size_t)25920 * 4096;
    for (const Sh &sh : shapes)
        if ((size_t)sh.M * sh.K > MA || (size_t)sh.N * sh.K > MW || (size_t)sh.M * sh.N > MO || sh.K % 128 || sh.N % 64) {
            printf("bad shape %s\n", sh.name);
            return 1;
        }
    int8_t *Aq, *Wq; float *Ad, *o1, *o2; uint16_t *Wd;
    CK(hipMalloc(&Aq, MA)); CK(hipMalloc(&Wq, MW)); CK(hipMalloc(&Ad, MA / 32 * 4)); CK(hipMalloc(&Wd, MW / 32 * 2));
    CK(hipMalloc(&o1, MO * 4)); CK(hipMalloc(&o2, MO * 4));
    {
        unsigned x = 99u;
        auto rnd = [&] { x = x * 1664525u + 1013904223u; return x >> 8; };
        std::vector<int8_t> q(MA);
        for (auto &v : q) v = (int8_t)((int)(rnd() % 255) - 127);
        CK(hipMemcpy(Aq, q.data(), MA, hipMemcpyHostToDevice));
        CK(hipMemcpy(Wq, q.data() + 5, MW, hipMemcpyHostToDevice));
        std::vector<float> d(MA / 32);
        for (auto &v : d) v = (float)(_Float16)(0.002f + 0.0001f * (float)(rnd() % 100));
        CK(hipMemcpy(Ad, d.data(), d.size() * 4, hipMemcpyHostToDevice));
        std::vector<uint16_t> w(MW / 32);
        for (auto &v : w) { _Float16 h = (_Float16)(0.001f + 0.00005f * (float)(rnd() % 100)); memcpy(&v, &h, 2); }
        CK(hipMemcpy(Wd, w.data(), w.size() * 2, hipMemcpyHostToDevice));
    }
    // the fp16-MFMA form's operands: the same quants as fp16 values, W scales in fp32
    uint16_t *Ah, *Wh; float *Wd32;
    CK(hipMalloc(&Ah, MA * 2)); CK(hipMalloc(&Wh, MW * 2)); CK(hipMalloc(&Wd32, MW / 32 * 4));
    {
        std::vector<int8_t> q(MA);
        CK(hipMemcpy(q.data(), Aq, MA, hipMemcpyDeviceToHost));
        std::vector<_Float16> h(MA);
        for (size_t i = 0; i < MA; i++) h[i] = (_Float16)q[i];
        CK(hipMemcpy(Ah, h.data(), MA * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(q.data(), Wq, MW, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < MW; i++) h[i] = (_Float16)q[i];
        CK(hipMemcpy(Wh, h.data(), MW * 2, hipMemcpyHostToDevice));
        std::vector<uint16_t> d(MW / 32);
        CK(hipMemcpy(d.data(), Wd, d.size() * 2, hipMemcpyDeviceToHost));
        std::vector<float> f(MW / 32);
        for (size_t i = 0; i < f.size(); i++) { _Float16 x; memcpy(&x, &d[i], 2); f[i] = (float)x; }
        CK(hipMemcpy(Wd32, f.data(), f.size() * 4, hipMemcpyHostToDevice));
    }
    for (const Sh &sh : shapes) {
        GemmArgs g{};
        g.Aq = Aq; g.lda = sh.K; g.Ad = Ad; g.ldad = sh.K / 32; g.Wq = Wq; g.ldw = sh.K; g.Wd = Wd;
        g.M = sh.M; g.N = sh.N; g.K = sh.K; g.ldo = sh.N;
        g.A = Ah; g.W = Wh;
        const double ops = 2.0 * sh.M * sh.N * sh.K;
        printf("%s  M=%d N=%d K=%d\n", sh.name, sh.M, sh.N, sh.K);
        g.out_f32 = o1;
        const double us0 = timeit([&] { run_gemm_q8<128, 64, 2, EPI_F32>(g, s); }, s);
        printf("  %-22s %8.1f us %6.1f TOP/s\n", "regs 128x64 KS2", us0, ops / us0 * 1e-6);
        std::vector<float> ref((size_t)sh.M * sh.N), got((size_t)sh.M * sh.N);
        CK(hipMemcpy(ref.data(), o1, ref.size() * 4, hipMemcpyDeviceToHost));
        auto var = [&](auto launch, const char *name) {
            g.out_f32 = o2;
            CK(hipMemset(o2, 0x7f, (size_t)sh.M * sh.N * 4));
            const double us = timeit(launch, s);
            CK(hipMemcpy(got.data(), o2, got.size() * 4, hipMemcpyDeviceToHost));
            const bool same = memcmp(ref.data(), got.data(), ref.size() * 4) == 0;
            printf("  %-22s %8.1f us %6.1f TOP/s  %s\n", name, us, ops / us * 1e-6, same ? "bit-identical" : "DIFFERENT");
        };
        if (sh.N % 128 == 0) {
            var([&] { run_gemm_q8h<128, 128, 1, 4, EPI_F32, 2>(g, Wd32, s); }, "f16 MFMA 128x128 KS1 NB4 4w");
            var([&] { run_gemm_q8h<128, 128, 1, 3, EPI_F32, 4>(g, Wd32, s); }, "f16 MFMA 128x128 KS1 NB3 8w");
            var([&] { run_gemm_q8h<128, 128, 2, 2, EPI_F32, 4>(g, Wd32, s); }, "f16 MFMA 128x128 KS2 NB2 8w");
            var([&] { run_gemm_q8h<128, 128, 1, 4, EPI_F32, 4>(g, Wd32, s); }, "f16 MFMA 128x128 KS1 NB4 8w");
        }
        var([&] { run_gemm_q8h<128, 64, 1, 4, EPI_F32, 2>(g, Wd32, s); }, "f16 MFMA 128x64 KS1 NB4 4w");
        var([&] { run_gemm_q8_glds<128, 64, 2, 2, EPI_F32>(g, s); }, "glds KS2 NB2");
    }
    return 0;
}
