// gemm.hip -- fp16 MFMA GEMM (C = A W^T) with fused epilogues, plus the
// weight-streaming skinny GEMV used by the decode step.
//
// Numerics = ggml_mul_mat with F16 weights (SURVEY.md §8(a) numerics i, iv):
// activations rounded to fp16 (RNE), fp16 x fp16 products accumulated in
// fp32.  v_mfma_f32_16x16x32_f16 has exactly these input semantics; only
// the summation order differs from ggml's SIMD lanes.
//
// Tiling: 256 threads = 4 waves (2x2), wave tile (BM/2)x(BN/2) built from
// 16x16x32 MFMAs; K staged through LDS in 32-wide slabs (KS slabs per
// barrier) of 64-byte rows with the chunk swizzle c ^ ((row>>1)&3), which is
// conflict-free for the ds_read_b128 fragment reads (checked exhaustively
// over the four 16-lane groups).  Register-staged double buffering: the next
// tile's global loads are issued before the current tile's MFMAs.
//
// A operand modes: dense row-major, or an implicit im2col gather over the
// NHWC conv activations (3x3, stride 2, pad 1) so conv2/conv3 of the audio
// encoder never materialise im2col buffers (src/audio_encoder.cpp:116-128).
#include "gemm_epi.h"
#include "gemm8p.h"

namespace qasr {

template <int BM, int BN, int KS, int AMODE, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
    constexpr int FM = BM / 32, FN = BN / 32;
    constexpr int ROWS = BM + BN;
    constexpr int SLAB = ROWS * 32;            // halves per slab (A rows then W rows)
    constexpr int NCH = ROWS * KS * 4;         // 16-byte chunks per stage
    constexpr int CPT = (NCH + 255) / 256;     // chunks per thread
    __shared__ __attribute__((aligned(16))) uint16_t smem[2 * KS * SLAB];
    __shared__ int4 rowinfo[AMODE == AM_DENSE ? 1 : BM];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int M = g.M, K = g.K;

    if constexpr (AMODE != AM_DENSE) {
        for (int r = tid; r < BM; r += 256) {
            const int row = m0 + r;
            int4 info = make_int4(-1, 0, 0, 0);
            if (row < M) {
                const int c = find_chunk(g.row_start, g.n_chunks, row);
                const ChunkDesc cd = g.chunks[c];
                const int local = row - g.row_start[c];
                int oh, ow, base, Win;
                if constexpr (AMODE == AM_CONV2) {
                    ow = local % cd.W2; oh = local / cd.W2; base = cd.row1; Win = cd.W1;
                } else {
                    oh = local % 16; ow = local / 16; base = cd.row2; Win = cd.W2;
                }
                info = make_int4(base, 2 * oh - 1, 2 * ow - 1, Win);
            }
            rowinfo[r] = info;
        }
        __syncthreads();
    }

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    u32x4 stage[CPT];
    auto gload = [&](int k0) {
        // conv modes: a stage's KS*32 k values lie inside one 3x3 tap (the host
        // guarantees C % (32*KS) == 0), so the tap and its (kh, kw) are uniform
        // per stage -- no per-chunk division by C
        int tap = 0, kh = 0, kw = 0;
        if constexpr (AMODE != AM_DENSE) {
            tap = k0 / g.C;
            kh = tap / 3;
            kw = tap - kh * 3;
        }
#pragma unroll
        for (int t = 0; t < CPT; t++) {
            const int c = tid + t * 256;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (c < NCH) {
                const int q = c & 3, rs = c >> 2;
                const int s = rs / ROWS, r = rs - s * ROWS;
                const int k = k0 + s * 32 + q * 8;
                if (r < BM) {
                    const int row = m0 + r;
                    if constexpr (AMODE == AM_DENSE) {
                        if (row < M) v = *(const u32x4 *)(g.A + (long)row * g.lda + k);
                    } else {
                        const int4 ri = rowinfo[r];
                        if (ri.x >= 0) {
                            const int ic = k - tap * g.C;
                            const int ih = ri.y + kh, iw = ri.z + kw;
                            const int Hin = AMODE == AM_CONV2 ? 64 : 32;
                            if (ih >= 0 && ih < Hin && iw >= 0 && iw < ri.w)
                                v = *(const u32x4 *)(g.A + ((long)(ri.x + ih * ri.w + iw) * g.C + ic));
                        }
                    }
                } else {
                    const int n = n0 + r - BM;
                    v = *(const u32x4 *)(g.W + (long)n * g.ldw + k);
                }
            }
            stage[t] = v;
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int t = 0; t < CPT; t++) {
            const int c = tid + t * 256;
            if (c < NCH) {
                const int q = c & 3, rs = c >> 2;
                const int s = rs / ROWS, r = rs - s * ROWS;
                uint16_t *dst = smem + (buf * KS + s) * SLAB + r * 32 + ((q ^ ((r >> 1) & 3)) << 3);
                *(u32x4 *)dst = stage[t];
            }
        }
    };

    const int nk = K / (32 * KS);
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * 32 * KS);
#pragma unroll
        for (int s = 0; s < KS; s++) {
            const uint16_t *sl = smem + (cur * KS + s) * SLAB;
            half8 af[FM], bf[FN];
            const int q = lane >> 4;
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const int r = wr * (BM / 2) + i * 16 + (lane & 15);
                af[i] = *(const half8 *)(sl + r * 32 + ((q ^ ((r >> 1) & 3)) << 3));
            }
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int r = BM + wc * (BN / 2) + j * 16 + (lane & 15);
                bf[j] = *(const half8 *)(sl + r * 32 + ((q ^ ((r >> 1) & 3)) << 3));
            }
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int j = 0; j < FN; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }

    gemm_epilogue<BM, BN, EPI>(g, acc, m0, n0, wr, wc, lane);
}

// ---------------------------------------------------- LDS-DMA tiled GEMM
// The same tile, fragments, swizzle and epilogue as gemm_kernel, but the
// operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging
// registers, no ds_write pass) through an NB-deep ring of stages (KS 32-deep
// slabs each), NB - 1 stages in flight behind the one being multiplied; one raw
// barrier per stage after a counted vmcnt (each wave waits only for its own
// pieces of the stage it is about to read).  The swizzle is applied on the
// source side: lane l of a 1-KiB piece lands at row l>>2, chunk position l&3,
// and fetches chunk (l&3) ^ ((row>>1)&3) -- the position the fragment reads
// expect.  Rows past M and conv taps in the padding fetch a global zero line
// (LDS-DMA has no per-lane predicate).
typedef __attribute__((address_space(3))) void lds_void_g;
typedef __attribute__((address_space(1))) void glb_void_g;
__device__ __attribute__((aligned(64))) uint32_t g_zero_line[16];

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// WNW: waves along N (2: 4 waves in a 2 x 2 grid, each BM/2 x BN/2; 4: 8 waves
// in 2 x 4, each BM/2 x BN/4 -- the 256-row tiles, whose 128 KiB of stages leave
// one workgroup a CU)
template <int BM, int BN, int KS, int NB, int AMODE, int EPI, int WNW = 2>
__global__ __launch_bounds__(128 * WNW) void gemm_glds_kernel(GemmArgs g) {
    constexpr int NWAVE = 2 * WNW, NTHR = 64 * NWAVE;
    constexpr int FM = BM / 32, FN = BN / (16 * WNW);
    constexpr int ROWS = BM + BN;
    constexpr int SLAB = ROWS * 32;        // halves per 32-deep slab
    constexpr int RG = ROWS / 16;          // 1-KiB pieces per slab
    constexpr int NP = KS * RG;            // pieces per stage
    constexpr int NW = (NP + NWAVE - 1) / NWAVE;   // pieces per wave per stage (uniform: vmcnt counts)
    constexpr int PAD = NW * NWAVE - NP;   // dummy pieces (zero line -> a scratch KiB) keep it uniform
    static_assert(ROWS % 16 == 0, "16-row pieces");
    static_assert(NB >= 2 && NB <= 4 && (NB - 2) * NW < 64, "ring depth");
    constexpr int INFO = AMODE == AM_DENSE ? 0 : BM * 8;   // int4 row descriptors (conv modes)
    constexpr int SCR = PAD ? 512 : 0;
    __shared__ __attribute__((aligned(16))) uint16_t smem[NB * KS * SLAB + SCR + INFO];
    int4 *rowinfo = (int4 *)(smem + NB * KS * SLAB + SCR);

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid / WNW, wc = wid % WNW;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int M = g.M, K = g.K;

    if constexpr (AMODE != AM_DENSE) {
        for (int r = tid; r < BM; r += NTHR) {
            const int row = m0 + r;
            int4 info = make_int4(-1, 0, 0, 0);
            if (row < M) {
                const int c = find_chunk(g.row_start, g.n_chunks, row);
                const ChunkDesc cd = g.chunks[c];
                const int local = row - g.row_start[c];
                int oh, ow, base, Win;
                if constexpr (AMODE == AM_CONV2) {
                    ow = local % cd.W2; oh = local / cd.W2; base = cd.row1; Win = cd.W1;
                } else {
                    oh = local % 16; ow = local / 16; base = cd.row2; Win = cd.W2;
                }
                info = make_int4(base, 2 * oh - 1, 2 * ow - 1, Win);
            }
            rowinfo[r] = info;
        }
        __syncthreads();
    }

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int lrow = lane >> 2, lpos = lane & 3;
    auto issue = [&](int k0, int buf) {
        int tap = 0, kh = 0, kw = 0;
        if constexpr (AMODE != AM_DENSE) {   // one 3x3 tap per stage (host: C % (32*KS) == 0)
            tap = k0 / g.C;
            kh = tap / 3;
            kw = tap - kh * 3;
        }
#pragma unroll
        for (int p = 0; p < NW; p++) {
            const int i = wid + NWAVE * p;
            if (PAD && i >= NP) {   // wave-uniform
                __builtin_amdgcn_global_load_lds((glb_void_g *)g_zero_line, (lds_void_g *)(smem + NB * KS * SLAB), 16, 0, 0);
                continue;
            }
            const int s = i / RG, rg = i - s * RG;
            const int r = rg * 16 + lrow;
            const int k = k0 + s * 32 + ((lpos ^ ((r >> 1) & 3)) << 3);
            const uint16_t *src = (const uint16_t *)g_zero_line;
            if (rg * 16 < BM) {
                const int row = m0 + r;
                if constexpr (AMODE == AM_DENSE) {
                    if (row < M) src = g.A + (long)row * g.lda + k;
                } else {
                    const int4 ri = rowinfo[r];
                    const int ih = ri.y + kh, iw = ri.z + kw;
                    const int Hin = AMODE == AM_CONV2 ? 64 : 32;
                    if (ri.x >= 0 && ih >= 0 && ih < Hin && iw >= 0 && iw < ri.w)
                        src = g.A + ((long)(ri.x + ih * ri.w + iw) * g.C + (k - tap * g.C));
                }
            } else {
                src = g.W + (long)(n0 + r - BM) * g.ldw + k;
            }
            __builtin_amdgcn_global_load_lds((glb_void_g *)src, (lds_void_g *)(smem + (buf * KS + s) * SLAB + rg * 512), 16, 0,
                                             0);
        }
    };

    const int nk = K / (32 * KS);
#pragma unroll
    for (int st = 0; st < NB - 1; st++)
        if (st < nk) issue(st * 32 * KS, st);
    int buf = 0;
    for (int kt = 0; kt < nk; kt++) {
        // this wave's pieces of stage kt have landed once at most the later
        // stages' pieces are outstanding
        const int ahead = nk - 1 - kt;
        if constexpr (NB >= 4) {
            if (ahead >= 2) wait_vm<2 * NW>();
            else if (ahead == 1) wait_vm<NW>();
            else wait_vm<0>();
        } else if constexpr (NB == 3) {
            if (ahead >= 1) wait_vm<NW>();
            else wait_vm<0>();
        } else {
            wait_vm<0>();
        }
        asm volatile("s_barrier" ::: "memory");   // every wave's pieces landed; stage kt-1's readers done
        if (kt + NB - 1 < nk) {
            int nb = buf + NB - 1;
            if (nb >= NB) nb -= NB;
            issue((kt + NB - 1) * 32 * KS, nb);
        }
#pragma unroll
        for (int s = 0; s < KS; s++) {
            const uint16_t *sl = smem + (buf * KS + s) * SLAB;
            half8 af[FM], bf[FN];
            const int q = lane >> 4;
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const int r = wr * (BM / 2) + i * 16 + (lane & 15);
                af[i] = *(const half8 *)(sl + r * 32 + ((q ^ ((r >> 1) & 3)) << 3));
            }
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int r = BM + wc * (BN / WNW) + j * 16 + (lane & 15);
                bf[j] = *(const half8 *)(sl + r * 32 + ((q ^ ((r >> 1) & 3)) << 3));
            }
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int j = 0; j < FN; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (++buf == NB) buf = 0;
    }
    gemm_epilogue<BM, BN, EPI, WNW>(g, acc, m0, n0, wr, wc, lane);
}

template <int BM, int BN, int KS, int AMODE, int EPI>
static void run_gemm(const GemmArgs &g, hipStream_t s) {
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    hipLaunchKernelGGL((gemm_kernel<BM, BN, KS, AMODE, EPI>), grid, dim3(256), 0, s, g);
}

template <int BM, int BN, int KS, int NB, int AMODE, int EPI, int WNW = 2>
static void run_glds(const GemmArgs &g, hipStream_t s) {
    dim3 grid(g.N / BN, (g.M + BM - 1) / BM);
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, KS, NB, AMODE, EPI, WNW>), grid, dim3(128 * WNW), 0, s, g);
}

template <int AMODE, int EPI>
static void dispatch_tiles(const GemmArgs &g, hipStream_t s) {
    if constexpr (AMODE != AM_DENSE) {
        // round 5: the 8-phase tile over the implicit im2col (weights zero-padded to g.ldw = K
        // rounded up to 128; tools/micro/g8_bench.hip) for >= 2048 output rows
        if (g.M >= 2048 && g.N >= 256 && g.N % 32 == 0 && g.C % 8 == 0 && g.ldw % 128 == 0 && g.ldw >= g.K &&
            g.ldw - g.K < 128 && g.ldo16 % 4 == 0 && !g.regs_staged) {
            GemmArgs h = g;
            h.K = g.ldw;
            run_gemm8p<EPI, AMODE>(h, s);
            return;
        }
        // conv: K = 9*C, slab group must stay inside one tap -> C % (32*KS) == 0
        if (g.N == 480) {
            // all 480 output channels per block: the gathered A tile is read once
            // (N/96 = 5 re-reads of the im2col rows otherwise), W stays L2-resident
            if (g.regs_staged) run_gemm<64, 480, 1, AMODE, EPI>(g, s);
            else run_glds<64, 480, 1, 2, AMODE, EPI>(g, s);
        } else if (g.N % 96 == 0 && g.C % 96 == 0) {
            if (g.M >= 4096) run_gemm<128, 96, 3, AMODE, EPI>(g, s);
            else run_gemm<64, 96, 3, AMODE, EPI>(g, s);
        } else {
            run_gemm<64, 64, 1, AMODE, EPI>(g, s);
        }
    } else {
        // tiles per shape from tools/gemm_bench.hip (MI355X): large M -> 128x128
        // (one 32-deep slab per stage up to K = 1024); ~1.2k rows (a 92 s
        // clip) -> 64x64 with 4 slabs per stage for the narrow, deep
        // projections (N <= 1024), 96x64 for the wide ones (N >= 3072)
        // round 3 (tools/micro/glds_gemm_bench.hip, MI355X, us per launch): 256 x 256
        // tiles on 8 waves with a 3-stage ring for the large shapes whose N takes
        // them (64 x 30 s prefill dn 272 -> 222, qkv 388 -> 374); 128 x 128 on 8
        // waves, 4-stage ring, for the wide projections of one clip (~1.2k rows:
        // prefill gate/up 39.6 -> 29.4, qkv 27.3 -> 25.1, encoder fc1 22.6 -> 21.3,
        // encoder qkv 19.8 -> 18.9; the narrow deep ones stay on 64 x 64 x 4)
        // round 5 (tools/micro/g8_bench.hip, MI355X, us per launch at 64 x 30 s): the 256 x
        // 256 8-phase tile (gemm8p.h) for every >= 2048-row projection it takes --
        // prefill qkv 370 -> 280, o 167 -> 125, gate/up 510 -> 351, down 220 -> 166,
        // encoder fc1 383 -> 258, fc2 251 -> 176, qkv 219 -> 164
        const bool big = g.M >= 2048 && g.N % 128 == 0;
        if constexpr (EPI != EPI_ARGMAX) {
            if (g.M >= 2048 && g.N >= 256 && g.N % 32 == 0 && g.K % 128 == 0 && g.lda % 8 == 0 && g.ldw % 8 == 0 && g.ldo % 4 == 0 &&
                g.ldo16 % 4 == 0 && (!g.res || g.ldr % 4 == 0) && !g.regs_staged) {
                run_gemm8p<EPI>(g, s);
                return;
            }
        }
        if (big && !g.regs_staged && g.N % 256 == 0) {
            run_glds<256, 256, 1, 3, AMODE, EPI, 4>(g, s);
        } else if (big && !g.regs_staged) {   // LDS-DMA stages (tools/micro/glds_gemm_bench.hip: +5-10 %)
            run_glds<128, 128, 1, 2, AMODE, EPI>(g, s);
        } else if (!big && !g.regs_staged && g.N >= 2048 && g.N % 128 == 0 && g.K % 32 == 0) {
            run_glds<128, 128, 1, 3, AMODE, EPI, 4>(g, s);
        } else if (big && g.K % 64 == 0) {
            if (g.K <= 1024) run_gemm<128, 128, 1, AMODE, EPI>(g, s);
            else run_gemm<128, 128, 2, AMODE, EPI>(g, s);
        } else if (!big && g.N <= 1024 && g.K % 128 == 0 && g.K >= 2048) {
            run_gemm<64, 64, 4, AMODE, EPI>(g, s);
        } else if (!big && g.N >= 3072 && g.N % 64 == 0 && g.K % 64 == 0) {
            run_gemm<96, 64, 2, AMODE, EPI>(g, s);
        } else if (g.K % 64 == 0) {
            run_gemm<64, 64, 2, AMODE, EPI>(g, s);
        } else {
            run_gemm<64, 64, 1, AMODE, EPI>(g, s);
        }
    }
}

void launch_gemm(int amode, int epi, const GemmArgs &g, hipStream_t s) {
    if (g.M <= 0) return;
    switch (amode * 8 + epi) {
        case AM_DENSE * 8 + EPI_F32: dispatch_tiles<AM_DENSE, EPI_F32>(g, s); break;
        case AM_DENSE * 8 + EPI_GELU_F16: dispatch_tiles<AM_DENSE, EPI_GELU_F16>(g, s); break;
        case AM_DENSE * 8 + EPI_SWIGLU_F16: dispatch_tiles<AM_DENSE, EPI_SWIGLU_F16>(g, s); break;
        case AM_DENSE * 8 + EPI_ARGMAX: dispatch_tiles<AM_DENSE, EPI_ARGMAX>(g, s); break;
        case AM_DENSE * 8 + EPI_F16: dispatch_tiles<AM_DENSE, EPI_F16>(g, s); break;
        case AM_DENSE * 8 + EPI_SWIGLU_F32: dispatch_tiles<AM_DENSE, EPI_SWIGLU_F32>(g, s); break;
        case AM_CONV2 * 8 + EPI_GELU_F16: dispatch_tiles<AM_CONV2, EPI_GELU_F16>(g, s); break;
        case AM_CONV3 * 8 + EPI_GELU_F16: dispatch_tiles<AM_CONV3, EPI_GELU_F16>(g, s); break;
        default: note_declined("launch_gemm", amode, epi); break;
    }
}

// a (mode, epilogue) pair no dispatcher instantiates: recorded per host thread
// (each context is driven by one thread) and turned into an error by the
// engine after the stage that launched it (take_declined), never skipped silently
static thread_local std::string t_declined;
void note_declined(const char *what, int mode, int epi) {
    if (t_declined.empty())
        t_declined = std::string(what) + " has no kernel for mode " + std::to_string(mode) + " / epilogue " + std::to_string(epi);
}
bool take_declined(std::string *msg) {
    if (t_declined.empty()) return false;
    if (msg) *msg = t_declined;
    t_declined.clear();
    return true;
}

// ===================================================================== GEMV
// One wave per CPW output columns; every lane streams 16-byte pieces of the
// weight rows straight from HBM into VGPRs (no LDS round trip for W, cdna
// guide: "GEMV / M <= 16 decode weights"), x rows live in LDS as fp16.
// NK = ceil(K/512) sweeps of a 64-lane x 8-half window.  The first column
// group's weights are requested before the x prologue so the two HBM
// latencies overlap; the grid strides over column groups beyond 1024 blocks.
template <int EPI, int CPW, int MR, int NK>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs g) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];   // [MR][K]
    __shared__ double red[4][MR];
    __shared__ unsigned long long bestk[4][MR];
    constexpr int NR = EPI == EPI_SWIGLU_F16 ? 2 : 1;   // weight rows per output
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    trace_mark(g.trace, 0);
    stamp_start(g.stamp);
    const int K = g.K;
    const int ncg = (g.N + CPW - 1) / CPW;
    int cg = blockIdx.x * 4 + wid;
    half8 wv[2][CPW][NR][NK];   // double-buffered: group i+1 is in flight while group i computes
    // Unconditional loads through a bounds-checked buffer descriptor: rows past
    // N get an out-of-range offset and return zeros without a memory access.
    // (A conditional load makes hipcc wait vmcnt(0) at the branch join, which
    // would serialise the weight stream behind the x prologue / the compute.)
    const uint32_t wbytes = (uint32_t)((long)g.N * NR * K * 2);
    const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc((void *)g.W, (short)0, (int)wbytes, 0x00020000);
    auto wload = [&](auto bc, int cgi) {
        constexpr int b = decltype(bc)::value;
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int r = 0; r < NR; r++)
#pragma unroll
                for (int t = 0; t < NK; t++) {
                    const int o = cgi * CPW + c, k = min(t * 512 + lane * 8, K - 8);
                    long wrow = o;
                    if constexpr (EPI == EPI_SWIGLU_F16) wrow = 32L * (o >> 4) + (o & 15) + 16 * r;
                    const uint32_t off = o < g.N ? (uint32_t)((wrow * K + k) * 2) : wbytes;
                    wv[b][c][r][t] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(wsrd, off, 0, 2));   // nt
                }
    };
    wload(std::integral_constant<int, 0>{}, cg);
    // ---- prologue: x rows -> fp16 in LDS (optionally RMS-normalised); each
    //      thread owns 4 consecutive elements per 1024-wide pass, one vector load each
    constexpr int KP = (NK * 512 + 1023) / 1024;
    if (g.norm_w || g.x) {
        float xr[MR][KP][4];
        double ss[MR];
#pragma unroll
        for (int m = 0; m < MR; m++) {
            ss[m] = 0.0;
#pragma unroll
            for (int p = 0; p < KP; p++) {
                const int k = p * 1024 + tid * 4;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (m < g.M && k < K) {
                    if (g.embd_ids) {
                        const uint2 hv = *(const uint2 *)(g.embd + (long)g.embd_ids[m] * K + k);
                        v = make_float4(u16_to_f(hv.x & 0xffff), u16_to_f(hv.x >> 16), u16_to_f(hv.y & 0xffff), u16_to_f(hv.y >> 16));
                        if (g.x_store && blockIdx.x == 0) *(float4 *)(g.x_store + (long)m * g.ldx + k) = v;
                    } else {
                        v = *(const float4 *)(g.x + (long)m * g.ldx + k);
                    }
                }
                xr[m][p][0] = v.x; xr[m][p][1] = v.y; xr[m][p][2] = v.z; xr[m][p][3] = v.w;
                ss[m] += (double)(v.x * v.x);
                ss[m] += (double)(v.y * v.y);
                ss[m] += (double)(v.z * v.z);
                ss[m] += (double)(v.w * v.w);
            }
        }
        if (g.norm_w) {
#pragma unroll
            for (int m = 0; m < MR; m++) {
                const double t = wave_sum_d(ss[m]);
                if (lane == 0) red[wid][m] = t;
            }
            __syncthreads();
        }
#pragma unroll
        for (int m = 0; m < MR; m++) {
            float scale = 1.0f;
            if (g.norm_w) {
                const double tot = red[0][m] + red[1][m] + red[2][m] + red[3][m];
                scale = 1.0f / sqrtf((float)(tot / K) + g.eps);
            }
#pragma unroll
            for (int p = 0; p < KP; p++) {
                const int k = p * 1024 + tid * 4;
                if (k < K) {
                    uint16_t h4[4];
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        float v = xr[m][p][e];
                        if (g.norm_w) v = fmul_rn(fmul_rn(v, scale), g.norm_w[k + e]);
                        h4[e] = m < g.M ? f_to_u16(v) : (uint16_t)0;
                    }
                    *(uint2 *)(xs + m * K + k) = make_uint2(h4[0] | ((uint32_t)h4[1] << 16), h4[2] | ((uint32_t)h4[3] << 16));
                }
            }
        }
    } else {
        for (int k = tid * 8; k < K; k += 256 * 8)
#pragma unroll
            for (int m = 0; m < MR; m++)
                *(u32x4 *)(xs + m * K + k) = m < g.M ? *(const u32x4 *)(g.xh + (long)m * g.ldxh + k) : u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();

    unsigned long long best[MR];
#pragma unroll
    for (int m = 0; m < MR; m++) best[m] = 0ull;
    const int stride = gridDim.x * 4;
    auto process = [&](auto bc, int cgi) {
        constexpr int b = decltype(bc)::value;
        const int col0 = cgi * CPW;
        // bias / residual of this group's outputs requested ahead of the sums and the
        // stores: a load between two stores makes the later store wait for the earlier
        // one's write (vmcnt in issue order), one round trip per output column (round 6)
        float bvv[CPW], rvv[CPW][MR];
        if constexpr (EPI == EPI_F32 || EPI == EPI_F16) {
            const float *zero = (const float *)g8_zero_line;
#pragma unroll
            for (int c = 0; c < CPW; c++) {
                const int oc = min(col0 + c, g.N - 1);
                bvv[c] = *(g.bias ? g.bias + oc : zero);
                if constexpr (EPI == EPI_F32)
#pragma unroll
                    for (int m = 0; m < MR; m++) rvv[c][m] = *(g.res ? g.res + (long)min(m, g.M - 1) * g.ldr + oc : zero);
            }
        }
        float acc[CPW][NR][MR];
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int r = 0; r < NR; r++)
#pragma unroll
                for (int m = 0; m < MR; m++) acc[c][r][m] = 0.0f;
#pragma unroll
        for (int t = 0; t < NK; t++) {
            const int k = t * 512 + lane * 8;
            if (k >= K) break;
#pragma unroll
            for (int m = 0; m < MR; m++) {
                const half8 xv = *(const half8 *)(xs + m * K + k);
#pragma unroll
                for (int c = 0; c < CPW; c++)
#pragma unroll
                    for (int r = 0; r < NR; r++)
#pragma unroll
                        for (int e = 0; e < 8; e++) acc[c][r][m] = fmaf((float)wv[b][c][r][t][e], (float)xv[e], acc[c][r][m]);
            }
        }
#pragma unroll
        for (int c = 0; c < CPW; c++) {
            const int o = col0 + c;
#pragma unroll
            for (int m = 0; m < MR; m++) {
                float v[NR];
#pragma unroll
                for (int r = 0; r < NR; r++) v[r] = wave_sum(acc[c][r][m]);
                if (o >= g.N || m >= g.M) continue;
                if constexpr (EPI == EPI_ARGMAX) {
                    if (lane == 0 && g.out_f32) g.out_f32[(long)m * g.ldo + o] = v[0];
                    const unsigned long long key = argmax_key(v[0], o);
                    best[m] = key > best[m] ? key : best[m];
                } else if (lane == 0) {
                    if constexpr (EPI == EPI_SWIGLU_F16) {
                        g.out_f16[(long)m * g.ldo16 + o] = f_to_u16(silu_f(v[0]) * v[1]);
                    } else {
                        float y = v[0];
                        if (g.bias) y = fadd_rn(y, bvv[c]);
                        if constexpr (EPI == EPI_F16) {
                            g.out_f16[(long)m * g.ldo16 + o] = f_to_u16(y);
                        } else {
                            if (g.res) y = fadd_rn(y, rvv[c][m]);
                            g.out_f32[(long)m * g.ldo + o] = y;
                        }
                    }
                }
            }
        }
    };
    while (cg < ncg) {
        const int n1 = cg + stride;
        wload(std::integral_constant<int, 1>{}, n1);   // past the end: no memory access
        process(std::integral_constant<int, 0>{}, cg);
        if (n1 >= ncg) break;
        const int n2 = n1 + stride;
        wload(std::integral_constant<int, 0>{}, n2);
        process(std::integral_constant<int, 1>{}, n1);
        cg = n2;
    }
    if constexpr (EPI != EPI_ARGMAX) {
        if (g.trace) { __syncthreads(); trace_mark(g.trace, 1); }
    }
    if constexpr (EPI == EPI_ARGMAX) {
        if (lane == 0)
#pragma unroll
            for (int m = 0; m < MR; m++) bestk[wid][m] = best[m];
        __syncthreads();
        if (tid < MR && tid < g.M) {
            unsigned long long b = bestk[0][tid];
            for (int w = 1; w < 4; w++) b = bestk[w][tid] > b ? bestk[w][tid] : b;
            const unsigned long long old = atomicMax(g.amax + tid, b);
            asm volatile("" ::"v"(old));   // returned value used: the add has been performed at L2
        }
        if (g.done) {
            __shared__ int last, st;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) last = __hip_atomic_fetch_add(g.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
            __syncthreads();
            if (last) {
                if (tid == 0) st = *g.step;
                __syncthreads();
                if (tid < g.M) {
                    const unsigned long long k = __hip_atomic_load(g.amax + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const int id = argmax_key_idx(k);
                    g.tok_out[tid] = id;
                    g.hist[(long)tid * g.hist_stride + st + 1] = id;
                    g.pos[tid] += 1;
                    __hip_atomic_store(g.amax + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (tid == 0) {
                    *g.step = st + 1;
                    __hip_atomic_store(g.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    stamp_end(g.stamp);
}

// ================================================================ Q8_0 GEMV
// Decode projections with Q8_0 weights (int8 [N][K] + fp16 scales [N][K/32]).
// Prologue: x rows (optionally RMS-normalised, optionally gathered from the
// embedding) quantised per 32 values exactly like quantize_row_q8_0 into LDS
// (int8 + fp32 scale); 8 threads own one block, amax by xor-shuffles.  Each
// lane streams 16 int8 weights per sweep (NK sweeps of 1024); two lanes form a
// block: v_dot4_i32_i8 x4, pair sum, then fma(d_w * d_x, sumi) (ggml order).
template <int EPI, int CPW, int MR, int NK>
__global__ __launch_bounds__(256) void gemv_q8_kernel(GemvArgs g) {
    extern __shared__ __attribute__((aligned(16))) int8_t xq[];   // [MR][K] int8, then [MR][K/32] fp32 scales
    __shared__ double red[4][MR];
    constexpr int NR = EPI == EPI_SWIGLU_F32 ? 2 : 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    trace_mark(g.trace, 0);
    const int K = g.K, nb = K / 32;
    float *xd = (float *)(xq + MR * K);
    const int ncg = (g.N + CPW - 1) / CPW;
    int cg = blockIdx.x * 4 + wid;
    const int8_t *Wq = (const int8_t *)g.W;
    u32x4 wv[CPW][NR][NK];
    uint16_t wdv[CPW][NR][NK];
    auto wload = [&](int cgi) {
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int r = 0; r < NR; r++)
#pragma unroll
                for (int t = 0; t < NK; t++) {
                    const int o = min(cgi * CPW + c, g.N - 1), k = min(t * 1024 + lane * 16, K - 16);
                    long wrow = o;
                    if constexpr (EPI == EPI_SWIGLU_F32) wrow = 32L * (o >> 4) + (o & 15) + 16 * r;
                    wv[c][r][t] = __builtin_nontemporal_load((const u32x4 *)(Wq + wrow * K + k));
                    wdv[c][r][t] = g.Wd[wrow * nb + (k >> 5)];
                }
    };
    if (cg < ncg) wload(cg);
    // ---- prologue: each thread owns 4 consecutive elements per 1024-wide pass
    constexpr int KP = NK;
    {
        float xr[MR][KP][4];
        double ss[MR];
#pragma unroll
        for (int m = 0; m < MR; m++) {
            ss[m] = 0.0;
#pragma unroll
            for (int p = 0; p < KP; p++) {
                const int k = p * 1024 + tid * 4;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (m < g.M && k < K) {
                    if (g.embd_ids) {
                        const uint2 hv = *(const uint2 *)(g.embd + (long)g.embd_ids[m] * K + k);
                        v = make_float4(u16_to_f(hv.x & 0xffff), u16_to_f(hv.x >> 16), u16_to_f(hv.y & 0xffff), u16_to_f(hv.y >> 16));
                        if (g.x_store && blockIdx.x == 0) *(float4 *)(g.x_store + (long)m * g.ldx + k) = v;
                    } else {
                        v = *(const float4 *)(g.x + (long)m * g.ldx + k);
                    }
                }
                xr[m][p][0] = v.x; xr[m][p][1] = v.y; xr[m][p][2] = v.z; xr[m][p][3] = v.w;
                ss[m] += (double)(v.x * v.x);
                ss[m] += (double)(v.y * v.y);
                ss[m] += (double)(v.z * v.z);
                ss[m] += (double)(v.w * v.w);
            }
        }
        if (g.norm_w) {
#pragma unroll
            for (int m = 0; m < MR; m++) {
                const double t = wave_sum_d(ss[m]);
                if (lane == 0) red[wid][m] = t;
            }
            __syncthreads();
        }
#pragma unroll
        for (int m = 0; m < MR; m++) {
            float scale = 1.0f;
            if (g.norm_w) {
                const double tot = red[0][m] + red[1][m] + red[2][m] + red[3][m];
                scale = 1.0f / sqrtf((float)(tot / K) + g.eps);
            }
#pragma unroll
            for (int p = 0; p < KP; p++) {
                const int k = p * 1024 + tid * 4;
                float v[4], amax = 0.0f;
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    v[e] = xr[m][p][e];
                    if (g.norm_w && k < K) v[e] = fmul_rn(fmul_rn(v[e], scale), g.norm_w[k + e]);
                    if (m >= g.M) v[e] = 0.0f;
                    amax = fmaxf(amax, fabsf(v[e]));
                }
                // block of 32 = 8 consecutive lanes (quantize_row_q8_0)
                amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
                amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
                amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
                if (k < K) {
                    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
                    uint32_t u = 0;
#pragma unroll
                    for (int e = 0; e < 4; e++) u |= (uint32_t)(uint8_t)(int8_t)__builtin_rintf(fmul_rn(v[e], id)) << (8 * e);
                    *(uint32_t *)(xq + m * K + k) = u;
                    if ((tid & 7) == 0) xd[m * nb + (k >> 5)] = u16_to_f(f_to_u16(amax / 127.f));
                }
            }
        }
    }
    __syncthreads();

    for (; cg < ncg; cg += gridDim.x * 4) {
        const int col0 = cg * CPW;
        float acc[CPW][NR][MR];
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int r = 0; r < NR; r++)
#pragma unroll
                for (int m = 0; m < MR; m++) acc[c][r][m] = 0.0f;
#pragma unroll
        for (int t = 0; t < NK; t++) {
            const int k = t * 1024 + lane * 16;
            const bool ok = k < K;   // lane-uniform per pair: K % 32 == 0
            const int kk = ok ? k : 0;
#pragma unroll
            for (int m = 0; m < MR; m++) {
                const u32x4 xv = *(const u32x4 *)(xq + m * K + kk);
                const float dx = xd[m * nb + (kk >> 5)];
#pragma unroll
                for (int c = 0; c < CPW; c++)
#pragma unroll
                    for (int r = 0; r < NR; r++) {
                        int si = __builtin_amdgcn_sdot4((int)wv[c][r][t].x, (int)xv.x, 0, false);
                        si = __builtin_amdgcn_sdot4((int)wv[c][r][t].y, (int)xv.y, si, false);
                        si = __builtin_amdgcn_sdot4((int)wv[c][r][t].z, (int)xv.z, si, false);
                        si = __builtin_amdgcn_sdot4((int)wv[c][r][t].w, (int)xv.w, si, false);
                        si += __shfl_xor(si, 1, 64);   // the two halves of the 32-block
                        const float dd = fmul_rn(u16_to_f(wdv[c][r][t]), dx);
                        if (ok && !(lane & 1)) acc[c][r][m] = fmaf(dd, (float)si, acc[c][r][m]);
                    }
            }
        }
        const int nxt = cg + gridDim.x * 4;
        if (nxt < ncg) wload(nxt);
#pragma unroll
        for (int c = 0; c < CPW; c++) {
            const int o = col0 + c;
#pragma unroll
            for (int m = 0; m < MR; m++) {
                float v[NR];
#pragma unroll
                for (int r = 0; r < NR; r++) v[r] = wave_sum(acc[c][r][m]);
                if (o >= g.N || m >= g.M || lane != 0) continue;
                if constexpr (EPI == EPI_SWIGLU_F32) {
                    g.out_f32[(long)m * g.ldo + o] = silu_f(v[0]) * v[1];
                } else {
                    float y = v[0];
                    if (g.bias) y = fadd_rn(y, g.bias[o]);
                    if (g.res) y = fadd_rn(y, g.res[(long)m * g.ldr + o]);
                    g.out_f32[(long)m * g.ldo + o] = y;
                }
            }
        }
    }
    if (g.trace) { __syncthreads(); trace_mark(g.trace, 1); }
}

template <int EPI, int CPW, int MR, int NK>
static void run_gemv_q8(const GemvArgs &g, hipStream_t s) {
    const int per_block = 4 * CPW;
    int blocks = (g.N + per_block - 1) / per_block;
    if (blocks > 1024) blocks = 1024;
    const size_t lds = (size_t)MR * g.K + (size_t)MR * (g.K / 32) * 4;
    hipLaunchKernelGGL((gemv_q8_kernel<EPI, CPW, MR, NK>), dim3(blocks), dim3(256), lds, s, g);
}

template <int EPI, int CPW, int MR>
static void gemv_q8_nk(const GemvArgs &g, hipStream_t s) {
    const int nk = (g.K + 1023) / 1024;
    if (nk <= 1) run_gemv_q8<EPI, CPW, MR, 1>(g, s);
    else if (nk <= 2) run_gemv_q8<EPI, CPW, MR, 2>(g, s);
    else if (nk <= 3) run_gemv_q8<EPI, CPW, MR, 3>(g, s);
    else if (nk <= 4) run_gemv_q8<EPI, CPW, MR, 4>(g, s);
    else run_gemv_q8<EPI, CPW, MR, 8>(g, s);
}

template <int EPI, int MR>
static void gemv_q8_cpw(const GemvArgs &g, hipStream_t s) {
    if (g.N >= 2048) gemv_q8_nk<EPI, 2, MR>(g, s);
    else gemv_q8_nk<EPI, 1, MR>(g, s);
}

template <int EPI>
static void gemv_q8_mr(const GemvArgs &g, hipStream_t s) {
    if (g.M <= 1) gemv_q8_cpw<EPI, 1>(g, s);
    else if (g.M <= 2) gemv_q8_cpw<EPI, 2>(g, s);
    else if (g.M <= 4) gemv_q8_cpw<EPI, 4>(g, s);
    else gemv_q8_cpw<EPI, 8>(g, s);
}

template <int EPI, int CPW, int MR, int NK>
static void run_gemv(const GemvArgs &g, hipStream_t s) {
    const int per_block = 4 * CPW;
    int blocks = (g.N + per_block - 1) / per_block;
    if (blocks > 1024) blocks = 1024;   // 256 CUs x 4 resident workgroups, grid-stride beyond
    const size_t lds = (size_t)MR * g.K * 2;
    hipLaunchKernelGGL((gemv_kernel<EPI, CPW, MR, NK>), dim3(blocks), dim3(256), lds, s, g);
}

template <int EPI, int CPW, int MR>
static void gemv_nk(const GemvArgs &g, hipStream_t s) {
    const int nk = (g.K + 511) / 512;
    if (nk <= 1) run_gemv<EPI, CPW, MR, 1>(g, s);
    else if (nk <= 2) run_gemv<EPI, CPW, MR, 2>(g, s);
    else if (nk <= 4) run_gemv<EPI, CPW, MR, 4>(g, s);
    else if (nk <= 6) run_gemv<EPI, CPW, MR, 6>(g, s);
    else run_gemv<EPI, CPW, MR, 8>(g, s);
}

template <int EPI, int MR>
static void gemv_cpw(const GemvArgs &g, hipStream_t s) {
    // keep >= ~512 waves in flight: fewer columns per wave for narrow outputs
    if (g.N >= 8192) gemv_nk<EPI, 4, MR>(g, s);
    else if (g.N >= 2048) gemv_nk<EPI, 2, MR>(g, s);
    else gemv_nk<EPI, 1, MR>(g, s);
}

template <int EPI>
static void gemv_mr(const GemvArgs &g, hipStream_t s) {
    if (g.M <= 1) gemv_cpw<EPI, 1>(g, s);
    else if (g.M <= 2) gemv_cpw<EPI, 2>(g, s);
    else if (g.M <= 4) gemv_cpw<EPI, 4>(g, s);
    else gemv_cpw<EPI, 8>(g, s);
}

void launch_gemv(int epi, const GemvArgs &g, hipStream_t s) {
    if (g.M <= 0) return;
    if (launch_gemv1(epi, g, s)) return;
    if (g.Wd) {   // Q8_0 weights: fp32 x only
        switch (epi) {
            case EPI_F32: gemv_q8_mr<EPI_F32>(g, s); break;
            case EPI_SWIGLU_F32: gemv_q8_mr<EPI_SWIGLU_F32>(g, s); break;
            default: note_declined("launch_gemv (Q8_0)", 0, epi); break;
        }
        return;
    }
    switch (epi) {
        case EPI_F32: gemv_mr<EPI_F32>(g, s); break;
        case EPI_SWIGLU_F16: gemv_mr<EPI_SWIGLU_F16>(g, s); break;
        case EPI_ARGMAX: gemv_mr<EPI_ARGMAX>(g, s); break;
        case EPI_F16: gemv_mr<EPI_F16>(g, s); break;
        default: note_declined("launch_gemv", 0, epi); break;
    }
}

}  // namespace qasr
