// mel.hip -- batched log-mel front-end for gfx950.
//
// Restates src/mel_spectrogram.cpp:484-628 (Linux path) on the GPU:
// reflect pad 200 -> periodic Hann (fp64) -> fp64 DFT over 201 bins x 400
// taps -> |X|^2 -> fp64 mel dot (128 x 201) -> log10(max(s,1e-10)) ->
// per-clip max over the n/160 kept frames -> clamp(max-8) -> (v+4)/4.
//
// The reference's Linux path is a naive fp64 DFT, not an FFT.  We keep its
// exact products (host-precomputed twiddle table built with the reference's
// own angle expression, mel_dft_twiddles) and its sequential tap order per
// (frame, bin), so every fp64 intermediate follows the same FMA chain as the
// reference build (C++ under g++ -O3 -march=native contracts by default:
// re += a*cos -> fma, im -= a*sin -> fma(-a, sin, im), |X|^2 -> fma(re, re,
// im*im), the mel dot -> fma; this file is built with -ffp-contract=off, so
// every fma here is written out) -- parity is bit-level in practice, and the
// whole stage is a few microseconds per 30 s clip, far below the encoder.
//
// Layout: one workgroup = FPB consecutive frames of one clip.  The windows of
// the FPB frames are staged in LDS (coalesced PCM reads, reflect padding
// resolved on load); thread k < 201 owns DFT bin k for all FPB frames, so
// each twiddle load (coalesced across k) is reused FPB times.
#include "dev_common.h"
#include "kernels.h"

namespace qasr {

#define MEL_FPB 8
#define MEL_NB 201
#define MEL_FS 400

__global__ __launch_bounds__(256) void mel_power_kernel(const float *__restrict__ pcm, const MelClip *__restrict__ clips,
                                                        const int2 *__restrict__ blocks, const double2 *__restrict__ tw,
                                                        const double *__restrict__ hann, const float *__restrict__ filt,
                                                        double *__restrict__ tmp, unsigned long long *__restrict__ cmax) {
    __shared__ double win[MEL_FPB][MEL_FS];
    __shared__ double pw[MEL_FPB][MEL_NB + 1];
    __shared__ double red[4];
    const int2 bi = blocks[blockIdx.x];
    const MelClip c = clips[bi.x];
    const int f0 = bi.y;
    const int tid = threadIdx.x;
    const float *x = pcm + c.pcm_off;
    const int n = c.n;
    for (int idx = tid; idx < MEL_FPB * MEL_FS; idx += 256) {
        const int f = idx / MEL_FS, j = idx - f * MEL_FS;
        const int fr = f0 + f;
        double v = 0.0;
        if (fr < c.TF) {
            const int p = fr * 160 + j;          // index into the reflect-padded signal
            float s;
            if (p < 200) {
                const int src = 200 - p;
                s = src < n ? x[src] : 0.0f;
            } else if (p < n + 200) {
                s = x[p - 200];
            } else {
                const int src = n - 2 - (p - n - 200);
                s = src >= 0 ? x[src] : 0.0f;
            }
            v = hann[j] * (double)s;
        }
        win[f][j] = v;
    }
    __syncthreads();
    if (tid < MEL_NB) {
        double re[MEL_FPB], im[MEL_FPB];
#pragma unroll
        for (int f = 0; f < MEL_FPB; f++) { re[f] = 0.0; im[f] = 0.0; }
        for (int t = 0; t < MEL_FS; t++) {
            const double2 w = tw[t * MEL_NB + tid];
#pragma unroll
            for (int f = 0; f < MEL_FPB; f++) {
                const double a = win[f][t];
                re[f] = fma(a, w.x, re[f]);
                im[f] = fma(-a, w.y, im[f]);
            }
        }
#pragma unroll
        for (int f = 0; f < MEL_FPB; f++) pw[f][tid] = fma(re[f], re[f], im[f] * im[f]);   // as g++ contracts re*re + im*im
    }
    __syncthreads();
    double bmax = -1e300;
    for (int o = tid; o < 128 * MEL_FPB; o += 256) {
        const int j = o / MEL_FPB, f = o - j * MEL_FPB;
        const int fr = f0 + f;
        if (fr >= c.TF) continue;
        const float *fj = filt + j * MEL_NB;
        double s = 0.0;
        for (int k = 0; k < MEL_NB; k++) s = fma(pw[f][k], (double)fj[k], s);
        const double lv = log10(s > 1e-10 ? s : 1e-10);
        tmp[c.tmp_off + (long)j * c.TF + fr] = lv;
        if (fr < c.TF - 1) bmax = fmax(bmax, lv);   // max over the n_len = TF-1 kept frames
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bmax = fmax(bmax, __shfl_xor(bmax, o, 64));
    if ((tid & 63) == 0) red[tid >> 6] = bmax;
    __syncthreads();
    if (tid == 0) {
        double m = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
        if (m > -1e299) atomicMax(cmax + bi.x, dkey(m));
    }
}

__global__ __launch_bounds__(256) void mel_norm_kernel(const MelClip *__restrict__ clips, int n_clips,
                                                       const double *__restrict__ tmp,
                                                       const unsigned long long *__restrict__ cmax,
                                                       float *__restrict__ out) {
    const int b = blockIdx.y;
    if (b >= n_clips) return;
    const MelClip c = clips[b];
    const int T = c.TF - 1;
    const long total = 128L * T;
    const double mx = dkey_inv(cmax[b]) - 8.0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int j = (int)(i / T), fr = (int)(i - (long)j * T);
        double v = tmp[c.tmp_off + (long)j * c.TF + fr];
        if (v < mx) v = mx;
        v = (v + 4.0) / 4.0;
        out[c.out_off + i] = (float)v;
    }
}

void launch_mel(const float *pcm, const MelClip *clips, int n_clips, const int2 *blocks, int n_blocks,
                const double2 *tw, const double *hann, const float *filt, double *tmp, unsigned long long *cmax,
                float *out, hipStream_t s) {
    if (n_blocks > 0)
        hipLaunchKernelGGL(mel_power_kernel, dim3(n_blocks), dim3(256), 0, s, pcm, clips, blocks, tw, hann, filt, tmp, cmax);
    if (n_clips > 0) hipLaunchKernelGGL(mel_norm_kernel, dim3(64, n_clips), dim3(256), 0, s, clips, n_clips, tmp, cmax, out);
}

int mel_frames_per_block() { return MEL_FPB; }

}  // namespace qasr
