/*
 * qasr_oracle.c -- CPU restatement of the reference Qwen3-ASR hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see qasr_oracle.h).  Every function cites the
 * reference file:line it restates.  ggml CPU numerics are restated from
 * upstream ggml (not vendored in the reference: SURVEY.md §0.1, §8(c)).
 */
#define _GNU_SOURCE
#include "qasr_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#if defined(__F16C__) && defined(__FMA__) && defined(__AVX2__)
#include <immintrin.h>
#define QO_SIMD 1
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static int g_threads = 4;
void qo_set_threads(int n) { g_threads = n > 0 ? n : 1; }

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* ======================================================================
 * fp16 <-> fp32, round-to-nearest-even (ggml_compute_fp32_to_fp16 / F16C)
 * ====================================================================== */
uint16_t qo_f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) {                     /* inf / nan */
        if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((ax >> 13) & 0x3ffu));
        return (uint16_t)(sign | 0x7c00u);
    }
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);   /* overflow -> inf */
    if (ax < 0x38800000u) {                      /* result subnormal or zero */
        if (ax <= 0x33000000u) return (uint16_t)sign;            /* <= 2^-25 -> 0 (RNE tie to even) */
        /* |f| = mant * 2^(e-150); half subnormal unit = 2^-24 -> q = mant >> (126-e) */
        uint32_t e = ax >> 23;
        uint32_t mant = (ax & 0x7fffffu) | 0x800000u;
        uint32_t sh = 126u - e;                  /* 14..24 */
        uint32_t q = mant >> sh;
        uint32_t rem = mant & ((1u << sh) - 1u);
        uint32_t half = 1u << (sh - 1);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    /* normal */
    uint32_t h = ((ax - 0x38000000u) >> 13);     /* rebias exponent 127->15 */
    uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

float qo_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    uint32_t x;
    if (e == 0) {
        if (m == 0) { x = sign; }
        else {
            int sh = 0;
            while (!(m & 0x400u)) { m <<= 1; sh++; }
            m &= 0x3ffu;
            x = sign | ((uint32_t)(113 - sh) << 23) | (m << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

static inline float round_f16(float x) { return qo_f16_to_f32(qo_f32_to_f16(x)); }

/* ggml_vec_mad_f16's per-element step on F16C (x86): fp16(fmaf(x, v, y)) --
 * the fma rounded to fp32, then RNE to fp16 (two roundings) */
uint16_t qo_f16_mad_round2(uint16_t x, float v, uint16_t y) {
    return qo_f32_to_f16(fmaf(qo_f16_to_f32(x), v, qo_f16_to_f32(y)));
}

/* the same step rounded ONCE: RNE to fp16 of the exact x * v + y (QO_FA_V_ROUND1;
 * what a fused mixed-precision fma with an fp16 result computes).  x * v is
 * exact in double (11 + 24 significant bits); TwoSum gives the double sum's
 * error; the sum is then rounded to odd at fp32 precision (24 >= 11 + 2 bits,
 * so the final RNE to fp16 equals RNE of the exact value) */
/* f (finite) lies exactly half-way between two adjacent fp16 values */
static int f16_midpoint(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x477ff000u) return 0;                        /* rounds to inf */
    if (ax >= 0x38800000u) return (ax & 0x1fffu) == 0x1000u;  /* normal fp16 range */
    if (ax < 0x33000000u) return 0;
    if (ax == 0x33000000u) return 1;                        /* 2^-25 */
    const uint32_t sh = 126u - (ax >> 23);
    const uint32_t mant = (ax & 0x7fffffu) | 0x800000u;
    return (mant & ((1u << sh) - 1u)) == (1u << (sh - 1));
}

uint16_t qo_f16_mad_round1(uint16_t x, float v, uint16_t y) {
    const double p = (double)qo_f16_to_f32(x) * (double)v;
    const double a = qo_f16_to_f32(y);
    const double s = p + a;
    if (!isfinite(s)) return qo_f32_to_f16((float)s);
    float f = (float)s;
    /* rounding is monotone and fp16 midpoints are fp32 values: RNE16(RN24(RN53(exact)))
     * errs only where the intermediate lands exactly on a midpoint the exact value is not */
    if (!f16_midpoint(f)) return qo_f32_to_f16(f);
    const double bp = s - a;
    const double e = (p - bp) + (a - (s - bp));   /* s + e == p + a exactly */
    if (e != 0.0 || (double)f != s) {
        /* exact value strictly between two adjacent floats lo < hi: take the odd one */
        float lo, hi;
        if ((double)f == s) {
            lo = e > 0 ? f : nextafterf(f, -INFINITY);
            hi = e > 0 ? nextafterf(f, INFINITY) : f;
        } else if ((double)f < s) {
            lo = f;
            hi = nextafterf(f, INFINITY);
        } else {
            lo = nextafterf(f, -INFINITY);
            hi = f;
        }
        uint32_t bl;
        memcpy(&bl, &lo, 4);
        f = (bl & 1u) ? lo : hi;
    }
    return qo_f32_to_f16(f);
}

/* ======================================================================
 * Mel front-end
 * ====================================================================== */

/* src/mel_spectrogram.cpp:353-359 */
static float hz_to_mel(float hz) { return 2595.0f * log10f(1.0f + hz / 700.0f); }
static float mel_to_hz(float mel) { return 700.0f * (powf(10.0f, mel / 2595.0f) - 1.0f); }

/* src/mel_spectrogram.cpp:361-415: HTK mel scale, (n_fft+1)*hz/sr bin points,
 * triangular weights on integer k, slaney-style 2/(hz[m+2]-hz[m]) scaling. */
void qo_mel_filters(float *filters) {
    const int n_mels = QO_N_MEL, n_fft = QO_N_FFT, sr = 16000;
    const int nb = 1 + n_fft / 2;
    float fmax = sr / 2.0f, fmin = 0.0f;
    float mel_min = hz_to_mel(fmin), mel_max = hz_to_mel(fmax);
    float mel_pts[QO_N_MEL + 2], hz_pts[QO_N_MEL + 2], bin_pts[QO_N_MEL + 2];
    for (int i = 0; i < n_mels + 2; i++) mel_pts[i] = mel_min + (mel_max - mel_min) * i / (n_mels + 1);
    for (int i = 0; i < n_mels + 2; i++) hz_pts[i] = mel_to_hz(mel_pts[i]);
    for (int i = 0; i < n_mels + 2; i++) bin_pts[i] = (n_fft + 1) * hz_pts[i] / sr;
    for (int m = 0; m < n_mels; m++) {
        float left = bin_pts[m], center = bin_pts[m + 1], right = bin_pts[m + 2];
        for (int k = 0; k < nb; k++) {
            float w = 0.0f;
            if (k >= left && k <= center) w = (k - left) / (center - left);
            else if (k >= center && k <= right) w = (right - k) / (right - center);
            filters[m * nb + k] = w;
        }
    }
    for (int m = 0; m < n_mels; m++) {
        float enorm = 2.0f / (hz_pts[m + 2] - hz_pts[m]);
        for (int k = 0; k < nb; k++) filters[m * nb + k] *= enorm;
    }
}

/* src/mel_spectrogram.cpp:484-628 (the Linux, non-Accelerate branch):
 * reflect-pad 200, periodic Hann (fp64), naive fp64 DFT (201 bins x 400
 * taps), |X|^2, fp64 mel dot, log10(max(s,1e-10)); global max over the
 * n_len = n/160 kept frames; clamp at max-8; (v+4)/4 -> float. */
int qo_log_mel(const float *samples, int n_samples, const float *filters, float *out) {
    const int fs = QO_N_FFT, step = QO_HOP, pad = fs / 2, nb = QO_N_BINS;
    const int n_pad = n_samples + 2 * pad;
    const int total_frames = (n_pad - fs) / step + 1;
    const int n_len = total_frames - 1;
    if (!out) return n_len;

    float *xp = (float *)calloc((size_t)n_pad, sizeof(float));
    memcpy(xp + pad, samples, (size_t)n_samples * sizeof(float));
    for (int i = 0; i < pad; i++) {
        int src = pad - i;
        xp[i] = src < n_samples ? samples[src] : 0.0f;
    }
    for (int i = 0; i < pad; i++) {
        int src = n_samples - 2 - i;
        xp[n_samples + pad + i] = src >= 0 ? samples[src] : 0.0f;
    }
    double hann[QO_N_FFT];
    for (int i = 0; i < fs; i++) hann[i] = 0.5 * (1.0 - cos((2.0 * M_PI * i) / (fs + 0)));

    double *tmp = (double *)malloc((size_t)QO_N_MEL * total_frames * sizeof(double));
    #pragma omp parallel for schedule(dynamic, 4) num_threads(g_threads)
    for (int i = 0; i < total_frames; i++) {
        const int off = i * step;
        double win[QO_N_FFT], power[QO_N_BINS];
        for (int j = 0; j < fs; j++) win[j] = hann[j] * (double)xp[off + j];
        for (int k = 0; k < nb; k++) {
            double re = 0.0, im = 0.0;
            for (int n = 0; n < fs; n++) {
                double angle = 2.0 * M_PI * k * n / fs;
                re += win[n] * cos(angle);
                im -= win[n] * sin(angle);
            }
            power[k] = re * re + im * im;
        }
        for (int j = 0; j < QO_N_MEL; j++) {
            double sum = 0.0;
            for (int k = 0; k < nb; k++) sum += power[k] * (double)filters[j * nb + k];
            tmp[(size_t)j * total_frames + i] = log10(sum > 1e-10 ? sum : 1e-10);
        }
    }
    double mmax = -1e20;
    for (int j = 0; j < QO_N_MEL; j++)
        for (int i = 0; i < n_len; i++) {
            double v = tmp[(size_t)j * total_frames + i];
            if (v > mmax) mmax = v;
        }
    mmax -= 8.0;
    for (int j = 0; j < QO_N_MEL; j++)
        for (int i = 0; i < n_len; i++) {
            double v = tmp[(size_t)j * total_frames + i];
            if (v < mmax) v = mmax;
            v = (v + 4.0) / 4.0;
            out[(size_t)j * n_len + i] = (float)v;
        }
    free(tmp);
    free(xp);
    return n_len;
}

/* src/mel_spectrogram.cpp:130-221: RIFF walk, PCM16 only, channel mean. */
int qo_load_wav(const char *path, float *out, int max_n, int *sample_rate) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char id[4];
    uint32_t u32;
    if (fread(id, 1, 4, f) != 4 || memcmp(id, "RIFF", 4)) { fclose(f); return -1; }
    if (fread(&u32, 4, 1, f) != 1) { fclose(f); return -1; }
    if (fread(id, 1, 4, f) != 4 || memcmp(id, "WAVE", 4)) { fclose(f); return -1; }
    uint16_t fmt = 0, nch = 0, bps = 0;
    uint32_t sr = 0;
    for (;;) {
        uint32_t sz;
        if (fread(id, 1, 4, f) != 4 || fread(&sz, 4, 1, f) != 1) break;
        if (!memcmp(id, "fmt ", 4)) {
            uint32_t br; uint16_t ba;
            if (fread(&fmt, 2, 1, f) != 1 || fread(&nch, 2, 1, f) != 1 || fread(&sr, 4, 1, f) != 1 ||
                fread(&br, 4, 1, f) != 1 || fread(&ba, 2, 1, f) != 1 || fread(&bps, 2, 1, f) != 1) break;
            if (sz > 16) fseek(f, sz - 16, SEEK_CUR);
        } else if (!memcmp(id, "data", 4)) {
            if (fmt != 1 || bps != 16 || nch == 0) { fclose(f); return -1; }
            if (sample_rate) *sample_rate = (int)sr;
            int n = (int)(sz / (bps / 8) / nch);
            if (!out) { fclose(f); return n; }
            if (n > max_n) n = max_n;
            int16_t *raw = (int16_t *)malloc((size_t)n * nch * sizeof(int16_t));
            size_t got = fread(raw, sizeof(int16_t), (size_t)n * nch, f);
            (void)got;
            for (int i = 0; i < n; i++) {
                if (nch == 1) out[i] = raw[i] / 32768.0f;
                else {
                    float s = 0;
                    for (int c = 0; c < nch; c++) s += raw[i * nch + c];
                    out[i] = (s / nch) / 32768.0f;
                }
            }
            free(raw);
            fclose(f);
            return n;
        } else {
            fseek(f, sz, SEEK_CUR);
        }
    }
    fclose(f);
    return -1;
}

/* ======================================================================
 * ggml CPU op restatements
 * ====================================================================== */

/* ggml_vec_dot_f16: fp16 x fp16 products accumulated in fp32 SIMD lanes. */
static float dot_f16(const uint16_t *x, const uint16_t *y, int n) {
#ifdef QO_SIMD
    __m256 acc[4] = {_mm256_setzero_ps(), _mm256_setzero_ps(), _mm256_setzero_ps(), _mm256_setzero_ps()};
    int i = 0;
    for (; i + 32 <= n; i += 32) {
        for (int j = 0; j < 4; j++) {
            __m256 a = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i + 8 * j)));
            __m256 b = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i + 8 * j)));
            acc[j] = _mm256_fmadd_ps(a, b, acc[j]);
        }
    }
    acc[0] = _mm256_add_ps(acc[0], acc[2]);
    acc[1] = _mm256_add_ps(acc[1], acc[3]);
    acc[0] = _mm256_add_ps(acc[0], acc[1]);
    float t[8];
    _mm256_storeu_ps(t, acc[0]);
    double s = 0.0;
    for (int j = 0; j < 8; j++) s += t[j];
    for (; i < n; i++) s += (double)(qo_f16_to_f32(x[i]) * qo_f16_to_f32(y[i]));
    return (float)s;
#else
    double s = 0.0;
    for (int i = 0; i < n; i++) s += (double)(qo_f16_to_f32(x[i]) * qo_f16_to_f32(y[i]));
    return (float)s;
#endif
}

/* ggml_vec_mad_f16: y = fp16(fma(x, v, y)) per element (F16C: 8 lanes
 * cvtph -> fmadd -> cvtps RNE; the scalar tail the same ops one at a time) */
static void vec_mad_f16(uint16_t *y, const uint16_t *x, int n, float v) {
    int i = 0;
#ifdef QO_SIMD
    const __m256 vv = _mm256_set1_ps(v);
    for (; i + 8 <= n; i += 8) {
        const __m256 a = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i)));
        const __m256 b = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i)));
        _mm_storeu_si128((__m128i *)(y + i), _mm256_cvtps_ph(_mm256_fmadd_ps(b, vv, a), _MM_FROUND_TO_NEAREST_INT));
    }
#endif
    for (; i < n; i++) y[i] = qo_f16_mad_round2(x[i], v, y[i]);
}

/* QO_FA_V_ROUND1: vec_mad_f16 with one rounding per element */
static void vec_mad_f16_round1(uint16_t *y, const uint16_t *x, int n, float v) {
    for (int i = 0; i < n; i++) y[i] = qo_f16_mad_round1(x[i], v, y[i]);
}

/* ggml_vec_scale_f16: y = fp16(y * v) */
static void vec_scale_f16(uint16_t *y, int n, float v) {
    int i = 0;
#ifdef QO_SIMD
    const __m256 vv = _mm256_set1_ps(v);
    for (; i + 8 <= n; i += 8) {
        const __m256 a = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i)));
        _mm_storeu_si128((__m128i *)(y + i), _mm256_cvtps_ph(_mm256_mul_ps(a, vv), _MM_FROUND_TO_NEAREST_INT));
    }
#endif
    for (; i < n; i++) y[i] = qo_f32_to_f16(qo_f16_to_f32(y[i]) * v);
}

/* ggml_vec_dot_f32 (fp32 x fp32, fp32 lanes) */
static float dot_f32(const float *x, const float *y, int n) {
    float acc[16] = {0};
    int i = 0;
    for (; i + 16 <= n; i += 16)
        for (int j = 0; j < 16; j++) acc[j] += x[i + j] * y[i + j];
    double s = 0.0;
    for (int j = 0; j < 16; j++) s += acc[j];
    for (; i < n; i++) s += x[i] * y[i];
    return (float)s;
}

/* ---- Q8_0 (ggml block_q8_0: fp16 d + 32 x int8, 34 B; type id 8) ------
 * Activation side of ggml_mul_mat with Q8_0 weights (vec_dot_type Q8_0):
 * quantize_row_q8_0, x86 AVX2 path of ggml-cpu/arch/x86/quants.c (the build
 * the reference's Linux CPU path compiles): amax per 32 values, d = amax/127
 * stored fp16, q = round-half-even(x * (127/amax)).  (The generic C path
 * uses id = 1/d and roundf; ties differ only, documented in DESIGN.md.) */
static void quantize_row_q8(const float *x, int K, int8_t *q, uint16_t *d) {
    for (int b = 0; b < K / 32; b++) {
        const float *xb = x + 32 * b;
        float amax = 0.0f;
        for (int i = 0; i < 32; i++) amax = fmaxf(amax, fabsf(xb[i]));
        const float dd = amax / 127.f;
        d[b] = qo_f32_to_f16(dd);
        const float id = amax != 0.0f ? 127.f / amax : 0.0f;
        for (int i = 0; i < 32; i++) q[32 * b + i] = (int8_t)nearbyintf(xb[i] * id);
    }
}

/* ggml_vec_dot_q8_0_q8_0, AVX2 path: per block the exact int products are
 * summed in 8 lanes of 4 (mul_sum_i8_pairs_float), each lane fma'd with
 * d_w * d_x into an fp32 accumulator, then hsum_float_8. */
static float dot_q8(const uint8_t *wrow, const int8_t *qx, const uint16_t *dx, int K) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = 0; b < K / 32; b++) {
        const uint8_t *blk = wrow + 34 * b;
        const uint16_t dwh = (uint16_t)(blk[0] | (blk[1] << 8));
        const int8_t *qw = (const int8_t *)(blk + 2);
        const float d = qo_f16_to_f32(dwh) * qo_f16_to_f32(dx[b]);
        for (int j = 0; j < 8; j++) {
            int s = 0;
            for (int i = 4 * j; i < 4 * j + 4; i++) s += (int)qw[i] * (int)qx[32 * b + i];
            acc[j] = fmaf(d, (float)s, acc[j]);
        }
    }
    const float r0 = acc[0] + acc[4], r1 = acc[1] + acc[5], r2 = acc[2] + acc[6], r3 = acc[3] + acc[7];
    return (r0 + r2) + (r1 + r3);
}

static void mul_mat_q8(const float *x, int M, int K, const uint8_t *w, int N, const float *bias, float *y) {
    const int nb = K / 32;
    int8_t *xq = (int8_t *)malloc((size_t)M * K);
    uint16_t *xd = (uint16_t *)malloc((size_t)M * nb * sizeof(uint16_t));
    #pragma omp parallel for num_threads(g_threads)
    for (int m = 0; m < M; m++) quantize_row_q8(x + (size_t)m * K, K, xq + (size_t)m * K, xd + (size_t)m * nb);
    #pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int n = 0; n < N; n++) {
        const uint8_t *wr = w + (size_t)n * nb * 34;
        for (int m = 0; m < M; m++) {
            float v = dot_q8(wr, xq + (size_t)m * K, xd + (size_t)m * nb, K);
            if (bias) v = v + bias[n];
            y[(size_t)m * N + n] = v;
        }
    }
    free(xq);
    free(xd);
}

static void mul_mat_f16(const float *x, int M, int K, const uint16_t *w, int N, const float *bias, float *y);

/* a linear layer's weight in the model's linear weight type (F16 or Q8_0) */
static void mul_mat_w(const qo_model *m, const float *x, int M, int K, const uint16_t *w, int N, const float *bias,
                      float *y) {
    if (m->wtype == QO_TYPE_Q8_0) mul_mat_q8(x, M, K, (const uint8_t *)w, N, bias, y);
    else mul_mat_f16(x, M, K, w, N, bias, y);
}

/* ggml_mul_mat(W[N][K] f16, X[M][K] f32): X is converted to fp16 (RNE,
 * vec_dot_type of F16) and every output is an fp32-accumulated fp16 dot.
 * y[M][N] = X W^T (+ bias, a separate ggml_add -> one fp32 rounding). */
static void mul_mat_f16(const float *x, int M, int K, const uint16_t *w, int N,
                        const float *bias, float *y) {
    uint16_t *xh = (uint16_t *)malloc((size_t)M * K * sizeof(uint16_t));
    #pragma omp parallel for num_threads(g_threads)
    for (int i = 0; i < M * K; i++) xh[i] = qo_f32_to_f16(x[i]);
    #pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int n = 0; n < N; n++) {
        const uint16_t *wr = w + (size_t)n * K;
        for (int m = 0; m < M; m++) {
            float v = dot_f16(xh + (size_t)m * K, wr, K);
            if (bias) v = v + bias[n];
            y[(size_t)m * N + n] = v;
        }
    }
    free(xh);
}

/* ggml_norm (eps) followed by ggml_mul(w) and ggml_add(b). Sums in double
 * (ggml_vec_sum_f32 / ggml_vec_cvar_f32), scale = 1/sqrtf(var+eps). */
static void layer_norm(const float *x, int M, int D, const float *w, const float *b,
                       float eps, float *y) {
    #pragma omp parallel for num_threads(g_threads)
    for (int m = 0; m < M; m++) {
        const float *xr = x + (size_t)m * D;
        float *yr = y + (size_t)m * D;
        double sum = 0.0;
        for (int i = 0; i < D; i++) sum += (double)xr[i];
        float mean = (float)(sum / D);
        double sum2 = 0.0;
        for (int i = 0; i < D; i++) {
            float v = xr[i] - mean;
            yr[i] = v;
            sum2 += (double)(v * v);
        }
        float var = (float)(sum2 / D);
        float scale = 1.0f / sqrtf(var + eps);
        for (int i = 0; i < D; i++) {
            float v = yr[i] * scale;
            if (w) v = v * w[i];
            if (b) v = v + b[i];
            yr[i] = v;
        }
    }
}

/* ggml_rms_norm (eps) + ggml_mul(w): sum of squares in double. */
static void rms_norm(const float *x, int M, int D, const float *w, float eps, float *y) {
    for (int m = 0; m < M; m++) {
        const float *xr = x + (size_t)m * D;
        float *yr = y + (size_t)m * D;
        double sum = 0.0;
        for (int i = 0; i < D; i++) sum += (double)(xr[i] * xr[i]);
        float mean = (float)(sum / D);
        float scale = 1.0f / sqrtf(mean + eps);
        for (int i = 0; i < D; i++) {
            float v = xr[i] * scale;
            if (w) v = v * w[i];
            yr[i] = v;
        }
    }
}

/* ggml tanh-GELU: ggml_gelu_f32 and its fp16 lookup table (GGML_GELU_FP16):
 * y = fp16(gelu(fp16(x))) for -10 < x < 10, 0 for x <= -10, x for x >= 10. */
static float gelu_f32(float x) {
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    return 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
}
static uint16_t *g_gelu_lut;
static void gelu_lut_init(void) {
    if (g_gelu_lut) return;
    uint16_t *t = (uint16_t *)malloc(65536 * sizeof(uint16_t));
    for (int i = 0; i < 65536; i++) t[i] = qo_f32_to_f16(gelu_f32(qo_f16_to_f32((uint16_t)i)));
    g_gelu_lut = t;
}
static inline float gelu(float x, int flags) {
    if (flags & QO_GELU_EXACT) return gelu_f32(x);
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return qo_f16_to_f32(g_gelu_lut[qo_f32_to_f16(x)]);
}

/* ggml_silu_f32: x / (1 + exp(-x)) */
static inline float silu(float x) { return x / (1.0f + expf(-x)); }

/* ======================================================================
 * Audio encoder
 * ====================================================================== */

/* src/audio_encoder.cpp:12-22 */
static void sinusoidal_pe(float *pe, int n_ctx, int d) {
    const int half = d / 2;
    for (int pos = 0; pos < n_ctx; ++pos)
        for (int i = 0; i < half; ++i) {
            float div_term = expf(-logf(10000.0f) * i / (half - 1));
            float angle = pos * div_term;
            pe[pos * d + i] = sinf(angle);
            pe[pos * d + half + i] = cosf(angle);
        }
}

/* src/audio_encoder.cpp:304-310 */
static int chunk_out_len(int L) {
    L = (L - 1) / 2 + 1;
    L = (L - 1) / 2 + 1;
    L = (L - 1) / 2 + 1;
    return L;
}

int qo_enc_frames(int T) {
    int n = 0;
    for (int s = 0; s < T; s += 100) n += chunk_out_len((T - s) < 100 ? (T - s) : 100);
    return n;
}

/* ggml_conv_2d(k3, s2, p1, d1) as im2col(fp16) + mul_mat, + bias, + GELU.
 * in [IC][H][W] fp32 -> out [OC][OH][OW] fp32.  Weight [OC][IC][3][3] fp16. */
static void conv2d_s2(const float *in, int IC, int H, int W, const uint16_t *w,
                      const float *b, int OC, float *out, int *OHp, int *OWp, int flags) {
    const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
    const int KK = IC * 9;
    uint16_t *col = (uint16_t *)malloc((size_t)OH * OW * KK * sizeof(uint16_t));
    #pragma omp parallel for num_threads(g_threads)
    for (int p = 0; p < OH * OW; p++) {
        int oh = p / OW, ow = p % OW;
        uint16_t *c = col + (size_t)p * KK;
        for (int ic = 0; ic < IC; ic++)
            for (int kh = 0; kh < 3; kh++)
                for (int kw = 0; kw < 3; kw++) {
                    int ih = oh * 2 - 1 + kh, iw = ow * 2 - 1 + kw;
                    float v = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? in[((size_t)ic * H + ih) * W + iw] : 0.0f;
                    c[ic * 9 + kh * 3 + kw] = qo_f32_to_f16(v);
                }
    }
    #pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int oc = 0; oc < OC; oc++) {
        const uint16_t *wr = w + (size_t)oc * KK;
        for (int p = 0; p < OH * OW; p++) {
            float v = dot_f16(col + (size_t)p * KK, wr, KK);
            v = v + b[oc];
            out[(size_t)oc * OH * OW + p] = gelu(v, flags);
        }
    }
    free(col);
    *OHp = OH;
    *OWp = OW;
}

/* src/audio_encoder.cpp:85-160 + :348-409: per 100-frame chunk (last one
 * short, not padded): conv x3 -> [W][C*16] (feature c*16+h) -> conv_out ->
 * + sinusoidal PE restarting at position 0 in every chunk.
 * QO_ENC_NO_CHUNK (AudioEncoder::encode_no_chunk, src/audio_encoder.cpp:603-663):
 * one chunk over all T frames, PE positions 0 .. N-1. */
int qo_encode_conv(const qo_model *m, const float *mel, int T, float *out, int flags) {
    gelu_lut_init();
    const int C = m->conv_ch, D = m->d_model, NM = m->n_mel;
    const int CH = (flags & QO_ENC_NO_CHUNK) ? (T > 0 ? T : 1) : 100;
    int n_out = 0;
    for (int s = 0; s < T; s += CH) {
        /* ASR: the chunk on its own length.  Aligner: one batched graph over
         * chunks zero-padded to 100 frames (src/forced_aligner.cpp:633-698);
         * the short last chunk keeps chunk_out_len(true length) frames (:725-733). */
        const int Lv = (T - s) < CH ? (T - s) : CH;
        const int L = m->aligner ? CH : Lv;
        float *x0 = (float *)calloc((size_t)NM * L, sizeof(float));
        for (int mm = 0; mm < NM; mm++)
            for (int f = 0; f < Lv; f++) x0[mm * L + f] = mel[(size_t)mm * T + s + f];
        int H1, W1, H2, W2, H3, W3;
        float *x1 = (float *)malloc((size_t)C * ((NM - 1) / 2 + 1) * ((L - 1) / 2 + 1) * sizeof(float));
        conv2d_s2(x0, 1, NM, L, m->conv1_w, m->conv1_b, C, x1, &H1, &W1, flags);
        float *x2 = (float *)malloc((size_t)C * H1 * W1 * sizeof(float));
        conv2d_s2(x1, C, H1, W1, m->conv2_w, m->conv2_b, C, x2, &H2, &W2, flags);
        float *x3 = (float *)malloc((size_t)C * H2 * W2 * sizeof(float));
        conv2d_s2(x2, C, H2, W2, m->conv3_w, m->conv3_b, C, x3, &H3, &W3, flags);
        const int F = C * H3;
        float *feat = (float *)malloc((size_t)W3 * F * sizeof(float));
        for (int t = 0; t < W3; t++)
            for (int c = 0; c < C; c++)
                for (int h = 0; h < H3; h++) feat[(size_t)t * F + c * H3 + h] = x3[((size_t)c * H3 + h) * W3 + t];
        float *y = out + (size_t)n_out * D;
        const int Wk = chunk_out_len(Lv);   /* = W3 for the ASR */
        mul_mat_w(m, feat, Wk, F, m->conv_out_w, D, NULL, y);
        float *pe = (float *)malloc((size_t)W3 * D * sizeof(float));
        sinusoidal_pe(pe, W3, D);
        for (int i = 0; i < Wk * D; i++) y[i] += pe[i];
        n_out += Wk;
        free(pe); free(feat); free(x3); free(x2); free(x1); free(x0);
    }
    return n_out;
}

/* ggml_mul_mat(K, Q) (fp32), ggml_soft_max_ext(scale), ggml_mul_mat(V, P):
 * full bidirectional attention, no mask (src/audio_encoder.cpp:466-486). */
static void enc_attention_seg(const float *qkv_q, const float *qkv_k, const float *qkv_v, int N,
                              int D, int H, float *out);
/* The aligner's block-diagonal mask (-inf outside windows of 13 * 800/100 =
 * 104 frames, src/forced_aligner.cpp:737-766) makes each window attend only
 * to itself: softmax over a window == the full softmax with the -inf mask. */
static void enc_attention(const qo_model *m, const float *q, const float *k, const float *v, int N, int D, int H,
                          float *out) {
    const int win = m->aligner ? 104 : N;
    for (int s0 = 0; s0 < N; s0 += win) {
        const int n = (N - s0) < win ? (N - s0) : win;
        enc_attention_seg(q + (size_t)s0 * D, k + (size_t)s0 * D, v + (size_t)s0 * D, n, D, H, out + (size_t)s0 * D);
    }
}

static void enc_attention_seg(const float *qkv_q, const float *qkv_k, const float *qkv_v, int N,
                              int D, int H, float *out) {
    const int hd = D / H;
    const float scale = 1.0f / sqrtf((float)hd);
    #pragma omp parallel for collapse(2) schedule(dynamic, 8) num_threads(g_threads)
    for (int h = 0; h < H; h++)
        for (int i = 0; i < N; i++) {
            float *s = (float *)malloc((size_t)N * sizeof(float));
            float qv[256], kv[256];
            for (int d = 0; d < hd; d++) qv[d] = qkv_q[(size_t)i * D + h * hd + d];
            float mx = -INFINITY;
            for (int j = 0; j < N; j++) {
                for (int d = 0; d < hd; d++) kv[d] = qkv_k[(size_t)j * D + h * hd + d];
                float v = dot_f32(kv, qv, hd) * scale;
                s[j] = v;
                if (v > mx) mx = v;
            }
            double sum = 0.0;
            for (int j = 0; j < N; j++) {
                float e = expf(s[j] - mx);
                s[j] = e;
                sum += (double)e;
            }
            float inv = (float)(1.0 / sum);
            for (int j = 0; j < N; j++) s[j] *= inv;
            float acc[256];
            for (int d = 0; d < hd; d++) acc[d] = 0.0f;
            /* V is made contiguous along n_ctx: out[d] = sum_j V[j][d] * P[j] */
            for (int d = 0; d < hd; d++) {
                float a[16] = {0};
                int j = 0;
                for (; j + 16 <= N; j += 16)
                    for (int t = 0; t < 16; t++) a[t] += qkv_v[(size_t)(j + t) * D + h * hd + d] * s[j + t];
                double ss = 0.0;
                for (int t = 0; t < 16; t++) ss += a[t];
                for (; j < N; j++) ss += qkv_v[(size_t)j * D + h * hd + d] * s[j];
                acc[d] = (float)ss;
            }
            for (int d = 0; d < hd; d++) out[(size_t)i * D + h * hd + d] = acc[d];
            free(s);
        }
}

/* src/audio_encoder.cpp:411-555 */
int qo_encode(const qo_model *m, const float *mel, int T, float *out, int flags) {
    const int D = m->d_model, H = m->enc_heads, FF = m->enc_ffn, HID = m->hidden;
    const int N = (flags & QO_ENC_NO_CHUNK) ? chunk_out_len(T) : qo_enc_frames(T);
    float *x = (float *)malloc((size_t)N * D * sizeof(float));
    qo_encode_conv(m, mel, T, x, flags);
    float *cur = (float *)malloc((size_t)N * D * sizeof(float));
    float *q = (float *)malloc((size_t)N * D * sizeof(float));
    float *k = (float *)malloc((size_t)N * D * sizeof(float));
    float *v = (float *)malloc((size_t)N * D * sizeof(float));
    float *att = (float *)malloc((size_t)N * D * sizeof(float));
    float *ff = (float *)malloc((size_t)N * FF * sizeof(float));
    for (int il = 0; il < m->enc_layers; il++) {
        const qo_enc_layer *L = &m->enc[il];
        layer_norm(x, N, D, L->attn_norm_w, L->attn_norm_b, m->enc_eps, cur);
        mul_mat_w(m, cur, N, D, L->attn_q_w, D, L->attn_q_b, q);
        mul_mat_w(m, cur, N, D, L->attn_k_w, D, L->attn_k_b, k);
        mul_mat_w(m, cur, N, D, L->attn_v_w, D, L->attn_v_b, v);
        enc_attention(m, q, k, v, N, D, H, att);
        mul_mat_w(m, att, N, D, L->attn_out_w, D, L->attn_out_b, cur);
        for (size_t i = 0; i < (size_t)N * D; i++) x[i] = cur[i] + x[i];
        layer_norm(x, N, D, L->ffn_norm_w, L->ffn_norm_b, m->enc_eps, cur);
        mul_mat_w(m, cur, N, D, L->ffn_up_w, FF, L->ffn_up_b, ff);
        for (size_t i = 0; i < (size_t)N * FF; i++) ff[i] = gelu(ff[i], flags);
        mul_mat_w(m, ff, N, FF, L->ffn_down_w, D, L->ffn_down_b, cur);
        for (size_t i = 0; i < (size_t)N * D; i++) x[i] = cur[i] + x[i];
    }
    layer_norm(x, N, D, m->ln_post_w, m->ln_post_b, m->enc_eps, cur);
    mul_mat_w(m, cur, N, D, m->proj1_w, D, m->proj1_b, q);
    for (size_t i = 0; i < (size_t)N * D; i++) q[i] = gelu(q[i], flags);
    mul_mat_w(m, q, N, D, m->proj2_w, HID, m->proj2_b, out);
    free(ff); free(att); free(v); free(k); free(q); free(cur); free(x);
    return N;
}

/* ======================================================================
 * Text decoder
 * ====================================================================== */
struct qo_dec {
    const qo_model *m;
    int n_ctx, flags;
    uint16_t *kc, *vc;      /* [layer][n_ctx][n_kv_head][head_dim] fp16 (text_decoder.cpp:366-376) */
};

qo_dec *qo_dec_new(const qo_model *m, int n_ctx, int flags) {
    qo_dec *d = (qo_dec *)calloc(1, sizeof(qo_dec));
    d->m = m;
    d->n_ctx = n_ctx;
    d->flags = flags;
    size_t per = (size_t)m->dec_layers * n_ctx * m->n_kv_head * m->head_dim;
    d->kc = (uint16_t *)calloc(per, sizeof(uint16_t));
    d->vc = (uint16_t *)calloc(per, sizeof(uint16_t));
    return d;
}

void qo_dec_free(qo_dec *d) {
    if (!d) return;
    free(d->kc);
    free(d->vc);
    free(d);
}

/* ggml_rope_cache_init + rope_yarn (ext_factor 0, freq_scale 1, mscale 1):
 * theta_i = p * theta_scale^i built by iterated fp32 multiplication. */
static void rope_neox(float *x, int n_dims, int pos, float base) {
    const float theta_scale = powf(base, -2.0f / n_dims);
    float cache[512];
    float theta = (float)pos;
    for (int i0 = 0; i0 < n_dims; i0 += 2) {
        cache[i0] = cosf(theta);
        cache[i0 + 1] = sinf(theta);
        theta *= theta_scale;
    }
    for (int i0 = 0; i0 < n_dims; i0 += 2) {
        const int ic = i0 / 2;
        const float c = cache[i0], s = cache[i0 + 1];
        const float x0 = x[ic], x1 = x[ic + n_dims / 2];
        x[ic] = x0 * c - x1 * s;
        x[ic + n_dims / 2] = x0 * s + x1 * c;
    }
}

/* src/text_decoder.cpp:392-581 (build_graph) + :588-684 (forward_with_audio) */
/* decoder layer stack; returns the final hidden rows x[n_tokens][hidden]
 * (caller frees).  al_fa: the aligner's attention (ggml_flash_attn_ext on
 * K kept in fp32 -> Q in fp32 and fp32 dots, V cast to fp16,
 * src/forced_aligner.cpp:1041-1046) instead of the fp16 KV cache. */
static float *dec_stack(qo_dec *dd, const int32_t *tokens, int n_tokens, const float *audio,
                        int n_audio, int audio_start_pos, int n_past, int al_fa) {
    const qo_model *m = dd->m;
    const int HS = m->hidden, NH = m->n_head, NKV = m->n_kv_head, HD = m->head_dim, FF = m->dec_ffn;
    const int QD = NH * HD, KD = NKV * HD;
    const int n_kv = n_past + n_tokens;
    if (n_kv > dd->n_ctx || n_tokens <= 0) return NULL;
    const float scale = 1.0f / sqrtf((float)HD);

    float *x = (float *)malloc((size_t)n_tokens * HS * sizeof(float));
    /* ggml_get_rows(token_embd F16) -> F32 */
    for (int t = 0; t < n_tokens; t++)
        for (int i = 0; i < HS; i++)
            x[(size_t)t * HS + i] = qo_f16_to_f32(m->token_embd[(size_t)tokens[t] * HS + i]);
    /* audio splice (text_decoder.cpp:431-459): rows [pos0, pos0+n_audio) */
    if (audio && n_audio > 0 && audio_start_pos >= 0 && audio_start_pos + n_audio <= n_tokens)
        memcpy(x + (size_t)audio_start_pos * HS, audio, (size_t)n_audio * HS * sizeof(float));

    float *cur = (float *)malloc((size_t)n_tokens * HS * sizeof(float));
    float *q = (float *)malloc((size_t)n_tokens * QD * sizeof(float));
    float *k = (float *)malloc((size_t)n_tokens * KD * sizeof(float));
    float *v = (float *)malloc((size_t)n_tokens * KD * sizeof(float));
    float *att = (float *)malloc((size_t)n_tokens * QD * sizeof(float));
    float *g = (float *)malloc((size_t)n_tokens * FF * sizeof(float));
    float *u = (float *)malloc((size_t)n_tokens * FF * sizeof(float));

    for (int il = 0; il < m->dec_layers; il++) {
        const qo_dec_layer *L = &m->dec[il];
        uint16_t *kc = dd->kc + (size_t)il * dd->n_ctx * KD;
        uint16_t *vc = dd->vc + (size_t)il * dd->n_ctx * KD;
        rms_norm(x, n_tokens, HS, L->attn_norm, m->rms_eps, cur);
        mul_mat_w(m, cur, n_tokens, HS, L->attn_q, QD, NULL, q);
        mul_mat_w(m, cur, n_tokens, HS, L->attn_k, KD, NULL, k);
        mul_mat_w(m, cur, n_tokens, HS, L->attn_v, KD, NULL, v);
        for (int t = 0; t < n_tokens; t++) {
            for (int h = 0; h < NH; h++) {
                float *qh = q + (size_t)t * QD + h * HD;
                if (L->attn_q_norm) rms_norm(qh, 1, HD, L->attn_q_norm, m->rms_eps, qh);
                rope_neox(qh, HD, n_past + t, m->rope_theta);
            }
            for (int h = 0; h < NKV; h++) {
                float *kh = k + (size_t)t * KD + h * HD;
                if (L->attn_k_norm) rms_norm(kh, 1, HD, L->attn_k_norm, m->rms_eps, kh);
                rope_neox(kh, HD, n_past + t, m->rope_theta);
            }
            /* ggml_cpy f32 -> f16 into the cache view at n_past + t */
            for (int i = 0; i < KD; i++) {
                kc[(size_t)(n_past + t) * KD + i] = qo_f32_to_f16(k[(size_t)t * KD + i]);
                vc[(size_t)(n_past + t) * KD + i] = qo_f32_to_f16(v[(size_t)t * KD + i]);
            }
        }
        /* ggml_flash_attn_ext CPU one-chunk path: Q -> fp16, fp16 dot,
         * online softmax, causal mask (k <= n_past + q), GQA h -> h / (NH/NKV),
         * fp16 V accumulator (or fp32 under QO_FA_V_F32). */
        const int rep = NH / NKV;
        #pragma omp parallel for collapse(2) schedule(dynamic, 4) num_threads(g_threads)
        for (int t = 0; t < n_tokens; t++)
            for (int h = 0; h < NH; h++) {
                const int hk = h / rep;
                uint16_t qh[512];
                for (int d = 0; d < HD; d++) qh[d] = qo_f32_to_f16(q[(size_t)t * QD + h * HD + d]);
                float S = 0.0f, M = -INFINITY;
                float acc32[512];
                uint16_t acc16[512];
                for (int d = 0; d < HD; d++) { acc32[d] = 0.0f; acc16[d] = 0; }
                const int limit = n_past + t;
                uint16_t vtmp[512];
                for (int ic = 0; ic <= limit; ic++) {
                    float s;
                    const uint16_t *vr;
                    if (al_fa) {   /* n_past = 0: key/value rows of this call */
                        s = dot_f32(k + (size_t)ic * KD + hk * HD, q + (size_t)t * QD + h * HD, HD);
                        for (int d = 0; d < HD; d++) vtmp[d] = qo_f32_to_f16(v[(size_t)ic * KD + hk * HD + d]);
                        vr = vtmp;
                    } else {
                        s = dot_f16(kc + (size_t)ic * KD + hk * HD, qh, HD);
                        vr = vc + (size_t)ic * KD + hk * HD;
                    }
                    s = s * scale;
                    const float Mold = M;
                    float ms = 1.0f, vs = 1.0f;
                    if (s > M) {
                        M = s;
                        ms = expf(Mold - M);
                        if (dd->flags & QO_FA_V_F32) for (int d = 0; d < HD; d++) acc32[d] *= ms;
                        else vec_scale_f16(acc16, HD, ms);
                    } else {
                        vs = expf(s - M);
                    }
                    if (dd->flags & QO_FA_V_F32) for (int d = 0; d < HD; d++) acc32[d] += qo_f16_to_f32(vr[d]) * vs;
                    else if (dd->flags & QO_FA_V_ROUND1) vec_mad_f16_round1(acc16, vr, HD, vs);
                    else vec_mad_f16(acc16, vr, HD, vs);
                    S = S * ms + vs;
                }
                if (!(dd->flags & QO_FA_V_F32)) for (int d = 0; d < HD; d++) acc32[d] = qo_f16_to_f32(acc16[d]);
                const float Sinv = S == 0.0f ? 0.0f : 1.0f / S;
                for (int d = 0; d < HD; d++) att[(size_t)t * QD + h * HD + d] = acc32[d] * Sinv;
            }
        mul_mat_w(m, att, n_tokens, QD, L->attn_output, HS, NULL, cur);
        for (size_t i = 0; i < (size_t)n_tokens * HS; i++) x[i] = cur[i] + x[i];
        rms_norm(x, n_tokens, HS, L->ffn_norm, m->rms_eps, cur);
        mul_mat_w(m, cur, n_tokens, HS, L->ffn_gate, FF, NULL, g);
        mul_mat_w(m, cur, n_tokens, HS, L->ffn_up, FF, NULL, u);
        for (size_t i = 0; i < (size_t)n_tokens * FF; i++) g[i] = silu(g[i]) * u[i];
        mul_mat_w(m, g, n_tokens, FF, L->ffn_down, HS, NULL, cur);
        for (size_t i = 0; i < (size_t)n_tokens * HS; i++) x[i] = cur[i] + x[i];
    }
    free(u); free(g); free(att); free(v); free(k); free(q); free(cur);
    return x;
}

/* src/text_decoder.cpp:392-581 (build_graph) + :588-684 (forward_with_audio):
 * last row only (:564-566) -> RMSNorm -> tied LM head */
int qo_dec_forward(qo_dec *dd, const int32_t *tokens, int n_tokens, const float *audio,
                   int n_audio, int audio_start_pos, int n_past, float *logits) {
    const qo_model *m = dd->m;
    const int HS = m->hidden;
    float *x = dec_stack(dd, tokens, n_tokens, audio, n_audio, audio_start_pos, n_past, 0);
    if (!x) return -1;
    float *cur = (float *)malloc((size_t)HS * sizeof(float));
    rms_norm(x + (size_t)(n_tokens - 1) * HS, 1, HS, m->output_norm, m->rms_eps, cur);
    mul_mat_f16(cur, 1, HS, m->token_embd, m->vocab, NULL, logits);
    free(cur); free(x);
    return 0;
}

int qo_align_forward(const qo_model *m, const int32_t *tokens, int n_tokens, const float *audio, int n_audio,
                     int audio_start_pos, const int *rows, int n_rows, float *logits, int flags) {
    if (!m->aligner || !m->classify_w) return -1;
    const int HS = m->hidden;
    qo_dec *dd = qo_dec_new(m, n_tokens, flags);
    float *x = dec_stack(dd, tokens, n_tokens, audio, n_audio, audio_start_pos, 0, 1);
    qo_dec_free(dd);
    if (!x) return -1;
    float *sel = (float *)malloc((size_t)(n_rows > 0 ? n_rows : 1) * HS * sizeof(float));
    for (int i = 0; i < n_rows; i++)   /* output_norm, then the classify head (no bias) */
        rms_norm(x + (size_t)rows[i] * HS, 1, HS, m->output_norm, m->rms_eps, sel + (size_t)i * HS);
    if (n_rows > 0) mul_mat_f16(sel, n_rows, HS, m->classify_w, m->classify_num, NULL, logits);
    free(sel); free(x);
    return 0;
}



/* src/qwen3_asr.cpp:305-317 */
int32_t qo_argmax(const float *logits, int n) {
    int32_t best = 0;
    float mv = logits[0];
    for (int i = 1; i < n; i++)
        if (logits[i] > mv) { mv = logits[i]; best = i; }
    return best;
}

/* src/qwen3_asr.cpp:151-214 with an empty system prompt */
int qo_build_prompt(const qo_model *m, int n_audio, int32_t *ids) {
    const int P = n_audio + 15;
    if (!ids) return P;
    int p = 0;
    ids[p++] = 151644; ids[p++] = 8948; ids[p++] = 198;
    ids[p++] = 151645; ids[p++] = 198;
    ids[p++] = 151644; ids[p++] = 872; ids[p++] = 198;
    ids[p++] = m->audio_start_id;
    for (int i = 0; i < n_audio; i++) ids[p++] = m->audio_pad_id;
    ids[p++] = m->audio_end_id;
    ids[p++] = 151645; ids[p++] = 198; ids[p++] = 151644; ids[p++] = 77091; ids[p++] = 198;
    return p;
}

/* src/qwen3_asr.cpp:81-149 + :216-303 (decode_greedy) */
int qo_transcribe(const qo_model *m, const float *pcm, int n, int max_tokens, int ignore_eos,
                  int flags, int32_t *tokens, double *t_ms) {
    double t0 = now_ms();
    float filters[QO_N_MEL * QO_N_BINS];
    qo_mel_filters(filters);
    const int T = qo_log_mel(pcm, n, filters, NULL);
    float *mel = (float *)malloc((size_t)QO_N_MEL * (T > 0 ? T : 1) * sizeof(float));
    /* the reference mel stage is single-threaded (src/mel_spectrogram.cpp:569-601) */
    int saved = g_threads;
    g_threads = 1;
    qo_log_mel(pcm, n, filters, mel);
    g_threads = saved;
    double t1 = now_ms();
    const int N = qo_enc_frames(T);
    float *feat = (float *)malloc((size_t)(N > 0 ? N : 1) * m->hidden * sizeof(float));
    qo_encode(m, mel, T, feat, flags);
    double t2 = now_ms();
    const int P = qo_build_prompt(m, N, NULL);
    int32_t *ids = (int32_t *)malloc((size_t)P * sizeof(int32_t));
    qo_build_prompt(m, N, ids);
    qo_dec *d = qo_dec_new(m, P + max_tokens, flags);
    float *logits = (float *)malloc((size_t)m->vocab * sizeof(float));
    int nt = 0;
    int pos0 = -1;     /* first <|audio_pad|> (src/qwen3_asr.cpp:230-239) */
    for (int i = 0; i < P && pos0 < 0; i++) if (ids[i] == m->audio_pad_id) pos0 = i;
    if (pos0 < 0) {    /* "No audio_pad token found in input sequence" */
        free(logits); qo_dec_free(d); free(ids); free(feat); free(mel);
        return -1;
    }
    qo_dec_forward(d, ids, P, feat, N, pos0, 0, logits);
    int32_t tok = qo_argmax(logits, m->vocab);
    tokens[nt++] = tok;
    int n_past = P;
    while ((ignore_eos || tok != m->eos_id) && nt < max_tokens) {
        qo_dec_forward(d, &tok, 1, NULL, 0, -1, n_past, logits);
        tok = qo_argmax(logits, m->vocab);
        tokens[nt++] = tok;
        n_past++;
    }
    if (!ignore_eos && nt > 0 && tokens[nt - 1] == m->eos_id) nt--;
    double t3 = now_ms();
    if (t_ms) { t_ms[0] = t1 - t0; t_ms[1] = t2 - t1; t_ms[2] = t3 - t2; }
    free(logits); qo_dec_free(d); free(ids); free(feat); free(mel);
    return nt;
}
