// gemm8p.h -- the large encoder / prefill GEMMs (C = A W^T, M >= 2048 rows):
// a 256 x 256 output tile per workgroup of 8 waves, K in 64-deep tiles, eight
// phases per pair of K-tiles (MI355X guide §5, "The 256² 8-phase template").
//
// LDS (128 KiB, the kernel's only LDS object): eight [128][64] fp16 images --
// for each of two K-tile buffers, A rows 0-127 (A0), A rows 128-255 (A1), W rows
// 0-127 (B0), W rows 128-255 (B1); the four A images first, then the four W
// images, so every fragment read reaches its image by an immediate offset from
// one of four address registers -- with 128-B rows whose 16-B chunk c sits at chunk
// position c ^ ((r >> 1) & 7): conflict-free for the fragment reads
// (ds_read_b128 lane groups, MI355X_MICROARCH.md §LDS).  Every half-tile is
// filled by LDS-DMA (global_load_lds_dwordx4, two 1-KiB pieces per wave), the
// swizzle applied on the source address.
//
// Wave (wr, wc) of the 2 x 4 grid owns rows wr*64 + [0, 64) of both A halves and
// columns wc*32 + [0, 32) of both W halves: four 64 x 32 quadrants, each one
// phase of 16 MFMAs (v_mfma_f32_16x16x32_f16) over a K-tile:
//   phase 1  read B0, A0    MFMA (A0, B0)   issue the odd buffer's A1
//   phase 2  read B1        MFMA (A0, B1)   issue the even buffer's B0 (next pair)
//   phase 3  read A1        MFMA (A1, B0)   issue even A0
//   phase 4  --             MFMA (A1, B1)   issue even B1, vmcnt(6): odd buffer landed
//   phases 5-8: the same on the odd buffer (issues: even A1, odd B0, A0, B1;
//   phase 8's vmcnt(6) lands the even buffer).
// Three half-tiles stay in flight across every barrier (raw s_barrier, counted
// vmcnt, never __syncthreads() in the loop).  Wave group wr = 1 runs one barrier
// behind group 0 (the two barriers of a phase bracket its MFMAs), so one
// group's reads and DMA issues overlap the other's MFMAs.  Ordering rules
// (cdna_hip_programming.md §5): a buffer is read one phase after the vmcnt that
// retires it, and restaged one phase after its last read when the reading phase
// retired those reads before its first barrier (B0: lgkmcnt(8) after the 4 B
// reads), two phases after otherwise.
//
// AMODE AM_CONV2 / AM_CONV3: the audio encoder's 3x3 stride-2 convs as implicit
// GEMMs over NHWC fp16 activations (gemm_kernel's gather): K = (tap, channel),
// each lane's 16-B piece is 8 channels of one tap, so the tap / channel split is
// per lane (channels % 8 == 0); a lane keeps its 4 rows' input origin (chunk base
// row, 2oh - 1, 2ow - 1, input width) in 8 registers, and taps in the padding --
// or in K past 9 * C, up to the weights' zero-padded row length (K % 128 == 0) --
// fetch a zero line.
//
// Every accumulator takes its K in the order of gemm_kernel / gemm_glds_kernel
// (32-deep steps, k ascending) with the same MFMA, so the outputs are
// bit-identical to theirs.  A last row (column) tile that would run past M (N)
// is shifted back to end at M (N) and stores only the rows (columns) no earlier
// tile stored, so every DMA source row is a valid row at a uniform offset from
// one per-lane base.
#pragma once
#include "gemm_epi.h"

namespace qasr {

typedef __attribute__((address_space(3))) void lds_void_8p;
typedef __attribute__((address_space(1))) void glb_void_8p;

__device__ __attribute__((aligned(64))) uint32_t g8_zero_line[16];
constexpr int G8_EPI_NONE = 99;    // tools/micro/g8_bench.hip: no output stores
constexpr int G8_HALF = 128 * 64;   // halves per [128][64] image (16 KiB)
// image of half-tile hid (0 A0, 1 A1, 2 B0, 3 B1) of buffer buf, in halves
__device__ __forceinline__ constexpr int g8_img(int hid, int buf) { return ((hid >> 1) * 4 + buf * 2 + (hid & 1)) * G8_HALF; }

template <int N>
__device__ __forceinline__ void g8_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void g8_lgkmcnt() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void g8_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// acc[i][j][fm][fn]: row m0 + 128i + 64wr + 16fm + 4(lane>>4) + r, column
// n0 + 128j + 32wc + 16fn + (lane&15) (v_mfma_*_16x16x* C layout).  Each wave
// turns one 64 x 32 quadrant at a time into row-major fp32 in its own 8 KiB of
// the (by now idle) LDS -- ds_write_b32, 2-way on the write side, which costs
// nothing (MI355X_MICROARCH.md §LDS), conflict-free ds_read_b128 back -- then
// applies the epilogue to 4 consecutive columns a lane and stores 16 B (fp32) /
// 8 B (fp16) a lane: whole 128-B (64-B) row segments per 8 lanes, ~1.2-1.6x
// faster than element stores from the MFMA layout (tools/micro/g8_bench.hip).
// The residual rows of the next quadrant are requested before this one is
// transposed (their HBM latency off the store path; every row of a tile is < M,
// the host guarantees M >= 256).  Per-element arithmetic as gemm_epilogue.
template <int EPI, bool RESV, bool PEV, bool SHIFT>
__device__ __forceinline__ void g8_epilogue(const GemmArgs &g, floatx4 (&acc)[2][2][4][2], uint16_t *smem, int m0, int n0,
                                            int mlo, int nlo, int wr, int wc, int lane) {
    const int M = g.M;
    if constexpr (EPI == G8_EPI_NONE) {   // micro-benchmark only: the main loop without the stores
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 2; j++)
#pragma unroll
                for (int fm = 0; fm < 4; fm++) t += acc[i][j][fm][0][0] + acc[i][j][fm][1][3];
        if (t == 1234.5f) g.out_f32[0] = t;
        return;
    }
    constexpr bool SWIGLU = EPI == EPI_SWIGLU_F16 || EPI == EPI_SWIGLU_F32;
    float *st = (float *)smem + (wr * 4 + wc) * 2048;   // this wave's [64][32] fp32 quadrant
    const int lr0 = SWIGLU ? (lane >> 2) : (lane >> 3);   // this lane's first row of a quadrant
    floatx4 rcur[RESV ? 8 : 1], rnext[RESV ? 8 : 1];
    auto load_res = [&](floatx4 (&dst)[RESV ? 8 : 1], int q) {
        const int col = n0 + (q & 1) * 128 + wc * 32 + 4 * (lane & 7);
        const int r0 = m0 + (q >> 1) * 128 + wr * 64 + lr0;
#pragma unroll
        for (int it = 0; it < 8; it++) dst[it] = *(const floatx4 *)(g.res + (long)(r0 + 8 * it) * g.ldr + col);
    };
    if constexpr (RESV) load_res(rcur, 0);
    floatx4 bias2[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    if (!SWIGLU && g.bias)
#pragma unroll
        for (int j = 0; j < 2; j++) bias2[j] = *(const floatx4 *)(g.bias + n0 + j * 128 + wc * 32 + 4 * (lane & 7));
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = q >> 1, j = q & 1;
        if constexpr (RESV)
            if (q < 3) load_res(rnext, q + 1);
        const int c0 = n0 + j * 128 + wc * 32;   // this wave's 32-column group
        const int r0 = m0 + i * 128 + wr * 64;
        if (!SHIFT || c0 >= nlo) {                 // (a shifted last column tile leaves the first ones to its neighbour)
#pragma unroll
            for (int fm = 0; fm < 4; fm++)
#pragma unroll
                for (int fn = 0; fn < 2; fn++)
#pragma unroll
                    for (int r = 0; r < 4; r++) st[(fm * 16 + 4 * (lane >> 4) + r) * 32 + fn * 16 + (lane & 15)] = acc[i][j][fm][fn][r];
            if constexpr (SWIGLU) {
                // gate in columns [0,16), up in [16,32) (interleaved weight rows): 4 lanes a row
#pragma unroll
                for (int it = 0; it < 4; it++) {
                    const int lr = lr0 + 16 * it, row = r0 + lr;
                    const floatx4 gt = *(const floatx4 *)(st + lr * 32 + 4 * (lane & 3));
                    const floatx4 up = *(const floatx4 *)(st + lr * 32 + 16 + 4 * (lane & 3));
                    if (SHIFT && row < mlo) continue;
                    const long o = c0 / 2 + 4 * (lane & 3);
                    floatx4 v;
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = silu_f(gt[e]) * up[e];
                    if constexpr (EPI == EPI_SWIGLU_F32) {
                        *(floatx4 *)(g.out_f32 + (long)row * g.ldo + o) = v;
                    } else {
                        *(uint2 *)(g.out_f16 + (long)row * g.ldo16 + o) =
                            make_uint2(f_to_u16(v[0]) | ((uint32_t)f_to_u16(v[1]) << 16), f_to_u16(v[2]) | ((uint32_t)f_to_u16(v[3]) << 16));
                    }
                }
            } else {
                const int col = c0 + 4 * (lane & 7);
                if constexpr (EPI == EPI_GELU_F16 || EPI == EPI_F16) {
                    // four rows at a time (GELU: 16 table reads in flight, 32 spilled registers)
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        uint32_t h[4][4];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const int it = 4 * hh + u;
                            floatx4 v = *(const floatx4 *)(st + (lr0 + 8 * it) * 32 + 4 * (lane & 7));
#pragma unroll
                            for (int e = 0; e < 4; e++) {
                                const float x = g.bias ? fadd_rn(v[e], bias2[j][e]) : v[e];
                                const uint32_t b16 = f_to_u16(x);
                                if constexpr (EPI == EPI_GELU_F16) {
                                    // gelu_lut_bits with its selects as bit masks: a select on a
                                    // loaded value becomes a branch around the load (one wait each)
                                    const uint32_t t = g.gelu[b16];
                                    const uint32_t hi = 0u - (uint32_t)(x >= 10.0f), lo = 0u - (uint32_t)(x <= -10.0f);
                                    h[u][e] = ((t & ~hi) | (b16 & hi)) & ~lo;
                                } else {
                                    h[u][e] = b16;
                                }
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const int row = r0 + lr0 + 8 * (4 * hh + u);
                            if (SHIFT && row < mlo) continue;
                            *(uint2 *)(g.out_f16 + (long)row * g.ldo16 + col) =
                                make_uint2(h[u][0] | (h[u][1] << 16), h[u][2] | (h[u][3] << 16));
                        }
                    }
                } else {
#pragma unroll
                    for (int it = 0; it < 8; it++) {
                        const int row = r0 + lr0 + 8 * it;
                        floatx4 v = *(const floatx4 *)(st + (lr0 + 8 * it) * 32 + 4 * (lane & 7));
                        if (SHIFT && row < mlo) continue;
                        floatx4 pv = floatx4{0.f, 0.f, 0.f, 0.f};
                        if constexpr (PEV) pv = *(const floatx4 *)(g.pe + (long)g.pe_pos[row] * g.N + col);   // conv_out only
#pragma unroll
                        for (int e = 0; e < 4; e++) {
                            if (g.bias) v[e] = fadd_rn(v[e], bias2[j][e]);
                            if constexpr (PEV) v[e] = fadd_rn(v[e], pv[e]);
                            if constexpr (RESV) v[e] = fadd_rn(v[e], rcur[it][e]);
                        }
                        *(floatx4 *)(g.out_f32 + (long)row * g.ldo + col) = v;
                    }
                }
            }
        }
        if constexpr (RESV)
            if (q < 3)
#pragma unroll
                for (int it = 0; it < 8; it++) rcur[it] = rnext[it];
    }
}

// The epilogue in straight-line versions: with a runtime residual / PE / shifted-tile
// test inside, the compiler's wait analysis merged paths with different numbers of
// stores and put vmcnt(0) -- one store-to-ack round trip -- ahead of every store
// (round 6).  Each version issues its loads (bias at entry, residual one quadrant
// ahead, LUT entries four rows at a time) before the stores that precede their use.
// 64 x 30 s, same box (profiles/r6/g8_epilogue_pipeline_ab.txt): encode 41.8 -> 32.6 ms,
// prefill 70.1 -> 60.2, utterance set 9330 -> 10036-10063 RTFx; epilogue cost over the
// bare loop at prefill qkv 184 -> 94 us (fp32 out), f16 114 -> 44 (g8_epilogue_waits.txt).
template <int EPI>
__device__ __forceinline__ void g8_epilogue_any(const GemmArgs &g, floatx4 (&acc)[2][2][4][2], uint16_t *smem, int m0, int n0,
                                                int mlo, int nlo, int wr, int wc, int lane) {
    const bool shift = m0 != mlo || n0 != nlo;
    if constexpr (EPI == EPI_F32) {
        if (g.res) {
            if (g.pe) {
                if (shift) g8_epilogue<EPI, true, true, true>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
                else g8_epilogue<EPI, true, true, false>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
            } else {
                if (shift) g8_epilogue<EPI, true, false, true>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
                else g8_epilogue<EPI, true, false, false>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
            }
        } else {
            if (g.pe) {
                if (shift) g8_epilogue<EPI, false, true, true>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
                else g8_epilogue<EPI, false, true, false>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
            } else {
                if (shift) g8_epilogue<EPI, false, false, true>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
                else g8_epilogue<EPI, false, false, false>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
            }
        }
    } else {
        if (shift) g8_epilogue<EPI, false, false, true>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
        else g8_epilogue<EPI, false, false, false>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
    }
}

// grid: one workgroup per 256 x 256 tile, 1-D, ceil(N/256) * ceil(M/256); host
// guarantees M >= 256, N >= 256, K % 128 == 0, N % 32 == 0, EPI not EPI_ARGMAX;
// conv modes: C % 8 == 0, K >= 9 * C, weight rows zero beyond 9 * C
template <int EPI, int AMODE = AM_DENSE>
__global__ __launch_bounds__(512) void gemm8p_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) uint16_t smem[8 * G8_HALF];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;
    const int M = g.M, N = g.N;

    // bijective XCD remap: the blocks dispatched to one XCD take consecutive tiles,
    // column tiles fastest (they share the A row tile in that XCD's L2)
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, rm = nwg & 7;
    const int wg = (xcd < rm ? xcd * (q + 1) : rm * (q + 1) + (xcd - rm) * q) + (orig >> 3);
    const int ntn = (N + 255) >> 8;
    const int mlo = (wg / ntn) * 256, nlo = (wg % ntn) * 256;   // first row / column this tile stores
    const int m0 = min(mlo, M - 256), n0 = min(nlo, N - 256);    // the tile's origin

    // this lane's DMA sources: piece (wid + 8p) of a half-tile = rows 8wid + 64p + (lane>>3),
    // landing at chunk position lane&7, so it fetches chunk (lane&7) ^ ((row>>1)&7)
    const int prow = wid * 8 + (lane >> 3);
    const int pchk = ((lane & 7) ^ ((prow >> 1) & 7)) * 8;
    // rows h*128 + p*64 + prow of the tile for half h, piece p: uniform offsets from one base
    const int aoff = (m0 + prow) * g.lda + pchk, woff = (n0 + prow) * g.ldw + pchk;
    // conv modes, per row j of this lane's 4 [half * 2 + piece]: the input position of tap (0, 0)
    // in 16-B units (8 channels: int32 holds a batch's whole activation), and the row's input
    // width << 16 | bit t = tap t inside the image (bits 9..15 stay 0: the K-padding taps read the zero line)
    int rbase[AMODE == AM_DENSE ? 1 : 4], rinfo[AMODE == AM_DENSE ? 1 : 4];
    if constexpr (AMODE != AM_DENSE) {
        constexpr int Hin = AMODE == AM_CONV2 ? 64 : 32;
        const int C8 = g.C >> 3;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int row = m0 + (j >> 1) * 128 + (j & 1) * 64 + prow;
            const int c = find_chunk(g.row_start, g.n_chunks, row);
            const ChunkDesc cd = g.chunks[c];
            const int local = row - g.row_start[c];
            int oh, ow, cb, Win;
            if constexpr (AMODE == AM_CONV2) {
                ow = local % cd.W2; oh = local / cd.W2; cb = cd.row1; Win = cd.W1;
            } else {
                oh = local % 16; ow = local / 16; cb = cd.row2; Win = cd.W2;
            }
            int mask = 0;
#pragma unroll
            for (int t = 0; t < 9; t++) {
                const int ih = 2 * oh - 1 + t / 3, iw = 2 * ow - 1 + t % 3;
                mask |= (ih >= 0 && ih < Hin && iw >= 0 && iw < Win) << t;
            }
            rbase[j] = (cb + (2 * oh - 1) * Win + (2 * ow - 1)) * C8;
            rinfo[j] = (Win << 16) | mask;
        }
    }
    // half-tile id: 0 A0, 1 A1, 2 B0, 3 B1
    auto issue = [&](int hid, int buf, int kt) {
        const bool isa = hid < 2;
        if (AMODE != AM_DENSE && isa) {
            const int C8 = g.C >> 3, k = kt * 64 + pchk;       // this lane's first channel of the tile, as a K index
            const int tap = (int)((k + 0.5f) * (1.0f / g.C));   // exact: k < 2^16, C >= 8
            const int ic8 = (k - tap * g.C) >> 3, kh = (tap * 11) >> 5, kw = tap - 3 * kh;   // tap / 3 for tap <= 10
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const int j = (hid & 1) * 2 + p, info = rinfo[j];
                const int off = rbase[j] + (kh * (info >> 16) + kw) * C8 + ic8;   // tap <= 8 when used
                const bool ok = (info >> tap) & 1;                                 // 0 for tap >= 9 (K padding)
                const uint16_t *pa = g.A + 8 * (long)off;
                const uint16_t *src = ok ? pa : (const uint16_t *)g8_zero_line;
                __builtin_amdgcn_global_load_lds((glb_void_8p *)src, (lds_void_8p *)(smem + g8_img(hid, buf) + (wid + 8 * p) * 512),
                                                 16, 0, 0);
            }
            return;
        }
        const int ld = isa ? g.lda : g.ldw;
        const uint16_t *base = (isa ? g.A : g.W) + kt * 64 + (isa ? aoff : woff);
#pragma unroll
        for (int p = 0; p < 2; p++) {
            const uint16_t *src = base + (long)((hid & 1) * 128 + p * 64) * ld;
            __builtin_amdgcn_global_load_lds((glb_void_8p *)src, (lds_void_8p *)(smem + g8_img(hid, buf) + (wid + 8 * p) * 512), 16,
                                             0, 0);
        }
    };

    half8 a[4][2], b0[2][2], b1[2][2];
    auto rd_a = [&](int buf, int h) {
        const uint16_t *img = smem + g8_img(h, buf);
#pragma unroll
        for (int fm = 0; fm < 4; fm++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++) {
                const int r = wr * 64 + fm * 16 + (lane & 15), c = kk * 4 + (lane >> 4);
                a[fm][kk] = *(const half8 *)(img + r * 64 + ((c ^ ((r >> 1) & 7)) << 3));
            }
    };
    auto rd_b = [&](half8 (&b)[2][2], int buf, int h) {
        const uint16_t *img = smem + g8_img(2 + h, buf);
#pragma unroll
        for (int fn = 0; fn < 2; fn++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++) {
                const int r = wc * 32 + fn * 16 + (lane & 15), c = kk * 4 + (lane >> 4);
                b[fn][kk] = *(const half8 *)(img + r * 64 + ((c ^ ((r >> 1) & 7)) << 3));
            }
    };

    floatx4 acc[2][2][4][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int fm = 0; fm < 4; fm++)
#pragma unroll
                for (int fn = 0; fn < 2; fn++) acc[i][j][fm][fn] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto mma = [&](floatx4 (&c)[4][2], half8 (&b)[2][2]) {
        g8_lgkmcnt<0>();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; kk++)
#pragma unroll
            for (int fm = 0; fm < 4; fm++)
#pragma unroll
                for (int fn = 0; fn < 2; fn++) c[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[fm][kk], b[fn][kk], c[fm][fn], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    const int niter = g.K >> 7;   // pairs of 64-deep K-tiles
    // prologue: K-tile 0 whole into buffer 0, K-tile 1's B0, A0, B1 into buffer 1;
    // K-tile 0 landed once at most those three half-tiles are outstanding
    issue(2, 0, 0);
    issue(0, 0, 0);
    issue(3, 0, 0);
    issue(1, 0, 0);
    issue(2, 1, 1);
    issue(0, 1, 1);
    issue(3, 1, 1);
    g8_vmcnt<6>();
    g8_barrier();
    if (wr == 1) g8_barrier();   // group 1 runs one barrier behind

    auto iteration = [&](int it, auto last) {
        constexpr bool LAST = decltype(last)::value;
        const int ke = 2 * it, ko = ke + 1;
        // phase 1
        rd_b(b0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        rd_a(0, 0);
        issue(1, 1, ko);
        g8_lgkmcnt<8>();   // the 4 B0 reads (issued first) retired: B0 may be restaged next phase
        g8_barrier();
        mma(acc[0][0], b0);
        g8_barrier();
        // phase 2
        rd_b(b1, 0, 1);
        if (!LAST) issue(2, 0, ke + 2);
        g8_barrier();
        mma(acc[0][1], b1);
        g8_barrier();
        // phase 3
        rd_a(0, 1);
        if (!LAST) issue(0, 0, ke + 2);
        g8_barrier();
        mma(acc[1][0], b0);
        g8_barrier();
        // phase 4
        if (!LAST) {
            issue(3, 0, ke + 2);
            g8_vmcnt<6>();
        } else {
            g8_vmcnt<0>();
        }
        g8_barrier();
        mma(acc[1][1], b1);
        g8_barrier();
        // phase 5
        rd_b(b0, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
        rd_a(1, 0);
        if (!LAST) issue(1, 0, ke + 2);
        g8_lgkmcnt<8>();
        g8_barrier();
        mma(acc[0][0], b0);
        g8_barrier();
        // phase 6
        rd_b(b1, 1, 1);
        if (!LAST) issue(2, 1, ko + 2);
        g8_barrier();
        mma(acc[0][1], b1);
        g8_barrier();
        // phase 7
        rd_a(1, 1);
        if (!LAST) issue(0, 1, ko + 2);
        g8_barrier();
        mma(acc[1][0], b0);
        g8_barrier();
        // phase 8
        if (!LAST) {
            issue(3, 1, ko + 2);
            g8_vmcnt<6>();
        }
        g8_barrier();
        mma(acc[1][1], b1);
        g8_barrier();
    };
    for (int it = 0; it < niter - 1; it++) iteration(it, std::false_type{});
    iteration(niter - 1, std::true_type{});
    if (wr == 0) g8_barrier();   // balance group 1's extra barrier

    g8_epilogue_any<EPI>(g, acc, smem, m0, n0, mlo, nlo, wr, wc, lane);
}

template <int EPI, int AMODE = AM_DENSE>
static inline void run_gemm8p(const GemmArgs &g, hipStream_t s) {
    const int tiles = ((g.N + 255) / 256) * ((g.M + 255) / 256);
    hipLaunchKernelGGL((gemm8p_kernel<EPI, AMODE>), dim3(tiles), dim3(512), 0, s, g);
}

}  // namespace qasr
