// conv1_bench.hip -- conv1 (csrc/elementwise.hip, included directly) at the
// 64 x 30 s encoder shape: us per launch and output GB/s of the engine kernel
// and of the round-4 form (one dependent load / gather / store round per row,
// kept here), outputs compared bit for bit.
#include "../../qwen3-asr.cpp_amd/csrc/elementwise.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace qasr;

namespace qasr {
// the round-4 form
__global__ __launch_bounds__(256) void conv1_r4_kernel(const float *__restrict__ mel, const ChunkDesc *__restrict__ chunks,
                                                    const int *__restrict__ row1_start, int n_chunks, int rows1,
                                                    const uint16_t *__restrict__ w, const float *__restrict__ b,
                                                    const uint16_t *__restrict__ lut, int C, uint16_t *__restrict__ act1) {
    // grid (positions / 16, chunk): no row -> chunk search
    const ChunkDesc cd = chunks[blockIdx.y];
    const int nloc = 64 * cd.W1;
    const int loc0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4;
    const int lane = threadIdx.x & 63;
    if (loc0 >= nloc || lane * 8 >= C) return;
    const int oc0 = lane * 8;
    float wf[8][9];
    {
        const u32x4 *wp = (const u32x4 *)(w + oc0 * 9);   // 72 consecutive halves
        uint16_t wh[72];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const u32x4 v = wp[i];
#pragma unroll
            for (int e = 0; e < 4; e++) { wh[8 * i + 2 * e] = v[e] & 0xffffu; wh[8 * i + 2 * e + 1] = v[e] >> 16; }
        }
#pragma unroll
        for (int o = 0; o < 8; o++)
#pragma unroll
            for (int t = 0; t < 9; t++) wf[o][t] = u16_to_f(wh[o * 9 + t]);
    }
    const float4 b0 = *(const float4 *)(b + oc0), b1 = *(const float4 *)(b + oc0 + 4);
    const float bias[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    for (int r = 0; r < 4; r++) {
        const int local = loc0 + r;
        if (local >= nloc) break;
        const int row = cd.row1 + local;
        const int oh = local / cd.W1, ow = local - oh * cd.W1;
        float in[9];
#pragma unroll
        for (int kh = 0; kh < 3; kh++)
#pragma unroll
            for (int kw = 0; kw < 3; kw++) {
                const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;   // ih: mel bin, iw: frame in chunk
                float v = 0.0f;
                if (ih >= 0 && ih < 128 && iw >= 0 && iw < cd.Lv) v = mel[cd.mel_off + (long)ih * cd.T + iw];
                in[kh * 3 + kw] = h2f(f2h(v));
            }
        uint32_t packed[4];
#pragma unroll
        for (int o = 0; o < 8; o++) {
            double sd = 0.0;
#pragma unroll
            for (int t = 0; t < 9; t++) sd += (double)(in[t] * wf[o][t]);
            const float v = fadd_rn((float)sd, bias[o]);
            const uint32_t h = gelu_lut_bits(v, lut);
            if (o & 1) packed[o >> 1] |= h << 16; else packed[o >> 1] = h;
        }
        *(u32x4 *)(act1 + (long)row * C + oc0) = u32x4{packed[0], packed[1], packed[2], packed[3]};
    }
}
// diagnostic (timing only, not the product's values): no GELU gather
__global__ __launch_bounds__(256) void conv1_nolut_kernel(const float *__restrict__ mel, const ChunkDesc *__restrict__ chunks,
                                                    const int *__restrict__ row1_start, int n_chunks, int rows1,
                                                    const uint16_t *__restrict__ w, const float *__restrict__ b,
                                                    const uint16_t *__restrict__ lut, int C, uint16_t *__restrict__ act1) {
    static_assert(9 * CONV1_ROWS <= 64, "one tap per lane");
    // grid (positions / 16, chunk): no row -> chunk search
    const ChunkDesc cd = chunks[blockIdx.y];
    const int nloc = 64 * cd.W1;
    const int loc0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * CONV1_ROWS;
    const int lane = threadIdx.x & 63;
    if (loc0 >= nloc) return;   // wave-uniform
    float tap = 0.0f;
    if (lane < 9 * CONV1_ROWS) {
        const int r = lane / 9, t = lane - r * 9, kh = t / 3, kw = t - kh * 3;
        const int local = loc0 + r;
        if (local < nloc) {
            const int oh = local / cd.W1, ow = local - oh * cd.W1;
            const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;   // ih: mel bin, iw: frame in chunk
            if (ih >= 0 && ih < 128 && iw >= 0 && iw < cd.Lv) tap = mel[cd.mel_off + (long)ih * cd.T + iw];
        }
        tap = h2f(f2h(tap));
    }
    const bool active = lane * 8 < C;
    const int oc0 = active ? lane * 8 : 0;
    float wf[8][9];
    {
        const u32x4 *wp = (const u32x4 *)(w + oc0 * 9);   // 72 consecutive halves
        uint16_t wh[72];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const u32x4 v = wp[i];
#pragma unroll
            for (int e = 0; e < 4; e++) { wh[8 * i + 2 * e] = v[e] & 0xffffu; wh[8 * i + 2 * e + 1] = v[e] >> 16; }
        }
#pragma unroll
        for (int o = 0; o < 8; o++)
#pragma unroll
            for (int t = 0; t < 9; t++) wf[o][t] = u16_to_f(wh[o * 9 + t]);
    }
    const float4 b0 = *(const float4 *)(b + oc0), b1 = *(const float4 *)(b + oc0 + 4);
    const float bias[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    uint32_t hv[CONV1_ROWS][8];
#pragma unroll
    for (int r = 0; r < CONV1_ROWS; r++) {
        float in[9];
#pragma unroll
        for (int t = 0; t < 9; t++) in[t] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tap), r * 9 + t));
#pragma unroll
        for (int o = 0; o < 8; o++) {
            double sd = 0.0;
#pragma unroll
            for (int t = 0; t < 9; t++) sd += (double)(in[t] * wf[o][t]);
            hv[r][o] = f_to_u16(fadd_rn((float)sd, bias[o]));
        }
    }
#pragma unroll
    for (int r = 0; r < CONV1_ROWS; r++) {
        const int local = loc0 + r;
        if (!active || local >= nloc) continue;
        const u32x4 v = {hv[r][0] | hv[r][1] << 16, hv[r][2] | hv[r][3] << 16, hv[r][4] | hv[r][5] << 16, hv[r][6] | hv[r][7] << 16};
        *(u32x4 *)(act1 + (long)(cd.row1 + local) * C + oc0) = v;
    }
}


// candidate: lane l owns 4 channels (36 weights held as doubles), two waves a row set:
// each product an exact double FMA (fp16 x fp16 fits fp32 and double exactly, so
// fma(in, w, sd) == sd + (double)(in * w), one rounding) -- 9 FP64 ops an output
// instead of 9 converts + 9 adds
template <int R>
__global__ __launch_bounds__(256) void conv1_dw_kernel(const float *__restrict__ mel, const ChunkDesc *__restrict__ chunks,
                                                       const uint16_t *__restrict__ w, const float *__restrict__ b,
                                                       const uint16_t *__restrict__ lut, int C, uint16_t *__restrict__ act1) {
    static_assert(9 * R <= 64, "one tap per lane");
    const ChunkDesc cd = chunks[blockIdx.y];
    const int nloc = 64 * cd.W1;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int loc0 = (blockIdx.x * 2 + (wv >> 1)) * R;   // waves (2p, 2p+1): the same rows, channel halves
    if (loc0 >= nloc) return;
    double tap = 0.0;
    if (lane < 9 * R) {
        const int r = lane / 9, t = lane - r * 9, kh = t / 3, kw = t - kh * 3;
        const int local = loc0 + r;
        float v = 0.0f;
        if (local < nloc) {
            const int oh = local / cd.W1, ow = local - oh * cd.W1;
            const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;
            if (ih >= 0 && ih < 128 && iw >= 0 && iw < cd.Lv) v = mel[cd.mel_off + (long)ih * cd.T + iw];
        }
        tap = (double)h2f(f2h(v));
    }
    const int ch = (wv & 1) * 256 + lane * 4;
    const bool active = ch < C;
    const int oc0 = active ? ch : 0;
    double wd[4][9];
    {
        const uint2 *wp = (const uint2 *)(w + oc0 * 9);   // 36 halves, 8-B aligned (oc0 % 4 == 0)
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const uint2 v = wp[i];
            const uint16_t hh[4] = {(uint16_t)(v.x & 0xffffu), (uint16_t)(v.x >> 16), (uint16_t)(v.y & 0xffffu), (uint16_t)(v.y >> 16)};
#pragma unroll
            for (int e = 0; e < 4; e++) wd[(4 * i + e) / 9][(4 * i + e) % 9] = (double)u16_to_f(hh[e]);
        }
    }
    const float4 bb = *(const float4 *)(b + oc0);
    const float bias[4] = {bb.x, bb.y, bb.z, bb.w};
    uint32_t hv[R][4];
#pragma unroll
    for (int r = 0; r < R; r++) {
        double in[9];
#pragma unroll
        for (int t = 0; t < 9; t++) {
            const long long u = __builtin_bit_cast(long long, tap);
            const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffll), r * 9 + t), hi = __builtin_amdgcn_readlane((int)(u >> 32), r * 9 + t);
            in[t] = __builtin_bit_cast(double, ((long long)(unsigned)lo) | ((long long)hi << 32));
        }
#pragma unroll
        for (int o = 0; o < 4; o++) {
            double sd = 0.0;
#pragma unroll
            for (int t = 0; t < 9; t++) sd = __builtin_fma(in[t], wd[o][t], sd);
            hv[r][o] = gelu_lut_bits(fadd_rn((float)sd, bias[o]), lut);
        }
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int local = loc0 + r;
        if (!active || local >= nloc) continue;
        *(uint2 *)(act1 + (long)(cd.row1 + local) * C + oc0) = make_uint2(hv[r][0] | hv[r][1] << 16, hv[r][2] | hv[r][3] << 16);
    }
}
}  // namespace qasr

int main() {
    hipStream_t s; CK(hipStreamCreate(&s));
    const int clips = 64, T = 3000, C = 480, L = 100, nchk = T / L;
    const int W1 = (L + 1) / 2, n_chunks = clips * nchk, rows1 = n_chunks * 64 * W1;
    std::vector<ChunkDesc> cd(n_chunks);
    for (int c = 0; c < clips; c++)
        for (int k = 0; k < nchk; k++) {
            ChunkDesc &d = cd[c * nchk + k];
            memset(&d, 0, sizeof d);
            d.mel_off = (long)c * 128 * T + k * L; d.T = T; d.L = L; d.Lv = L; d.W1 = W1;
            d.row1 = (c * nchk + k) * 64 * W1;
        }
    float *mel, *b; uint16_t *w, *lut, *o1, *o2; ChunkDesc *dcd;
    CK(hipMalloc(&mel, (size_t)clips * 128 * T * 4)); CK(hipMalloc(&b, C * 4)); CK(hipMalloc(&w, C * 9 * 2));
    CK(hipMalloc(&lut, 65536 * 2)); CK(hipMalloc(&o1, (size_t)rows1 * C * 2)); CK(hipMalloc(&o2, (size_t)rows1 * C * 2));
    CK(hipMalloc(&dcd, n_chunks * sizeof(ChunkDesc)));
    CK(hipMemcpy(dcd, cd.data(), n_chunks * sizeof(ChunkDesc), hipMemcpyHostToDevice));
    {
        unsigned x = 7u;
        auto rnd = [&] { x = x * 1664525u + 1013904223u; return (float)(x >> 8) / 16777216.0f; };
        std::vector<float> m((size_t)clips * 128 * T);
        for (auto &v : m) v = rnd() * 4.0f - 2.0f;
        CK(hipMemcpy(mel, m.data(), m.size() * 4, hipMemcpyHostToDevice));
        std::vector<_Float16> wh(C * 9);
        for (auto &v : wh) v = (_Float16)(rnd() - 0.5f);
        CK(hipMemcpy(w, wh.data(), wh.size() * 2, hipMemcpyHostToDevice));
        std::vector<float> bb(C);
        for (auto &v : bb) v = rnd() * 0.2f - 0.1f;
        CK(hipMemcpy(b, bb.data(), C * 4, hipMemcpyHostToDevice));
        std::vector<uint16_t> l(65536);
        for (int i = 0; i < 65536; i++) l[i] = (uint16_t)(i * 2654435761u >> 16);
        CK(hipMemcpy(lut, l.data(), l.size() * 2, hipMemcpyHostToDevice));
    }
    const int per_block = 16, max_loc = 64 * W1;   // the round-4 form: 4 rows a wave
    auto old_launch = [&] {
        hipLaunchKernelGGL(conv1_r4_kernel, dim3((max_loc + per_block - 1) / per_block, n_chunks), dim3(256), 0, s, mel, dcd,
                           nullptr, n_chunks, rows1, w, b, lut, C, o1);
    };
    auto new_launch = [&] { launch_conv1(mel, dcd, nullptr, n_chunks, rows1, w, b, lut, C, o2, s, W1); };
    auto timeit = [&](auto f) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        f(); CK(hipStreamSynchronize(s));
        float best = 1e30f;
        for (int it = 0; it < 5; it++) {
            CK(hipEventRecord(e0, s)); f(); CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;
        }
        return best;
    };
    const double bytes = (double)rows1 * C * 2;
    const float t0 = timeit(old_launch), t1 = timeit(new_launch);
    std::vector<uint16_t> h1((size_t)rows1 * C), h2((size_t)rows1 * C);
    CK(hipMemcpy(h1.data(), o1, h1.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), o2, h2.size() * 2, hipMemcpyDeviceToHost));
    const bool same = memcmp(h1.data(), h2.data(), h1.size() * 2) == 0;
    const float t2 = timeit([&] {
        hipLaunchKernelGGL(conv1_nolut_kernel, dim3((max_loc + 4 * CONV1_ROWS - 1) / (4 * CONV1_ROWS), n_chunks), dim3(256), 0, s, mel, dcd,
                           nullptr, n_chunks, rows1, w, b, lut, C, o1);
    });
    printf("  (diagnostic: the engine kernel without the GELU gather %.3f ms, %.2f TB/s)\n", t2, bytes / t2 * 1e-9);
    auto dw = [&](auto kernel, int R, const char *name) {
        CK(hipMemset(o1, 0, (size_t)rows1 * C * 2));
        const float t = timeit([&] {
            hipLaunchKernelGGL(kernel, dim3((max_loc + 2 * R - 1) / (2 * R), n_chunks), dim3(256), 0, s, mel, dcd, w, b, lut, C, o1);
        });
        CK(hipMemcpy(h1.data(), o1, h1.size() * 2, hipMemcpyDeviceToHost));
        const bool eq = memcmp(h1.data(), h2.data(), h1.size() * 2) == 0;
        printf("  %s: %.3f ms (%.2f TB/s) %s\n", name, t, bytes / t * 1e-9, eq ? "bit-identical" : "DIFFERENT");
    };
    dw(conv1_dw_kernel<4>, 4, "double-weight FMA form, 4 rows a wave");
    dw(conv1_dw_kernel<7>, 7, "double-weight FMA form, 7 rows a wave");
    printf("conv1 64 x 30 s, %d rows a wave (%d rows x %d ch, %.2f GB out): round-4 form %.3f ms (%.2f TB/s), engine %.3f ms (%.2f TB/s), %s\n", CONV1_ROWS,
           rows1, C, bytes * 1e-9, t0, bytes / t0 * 1e-9, t1, bytes / t1 * 1e-9, same ? "bit-identical" : "DIFFERENT");
    return same ? 0 : 1;
}
