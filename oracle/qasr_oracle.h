/*
 * qasr_oracle.h -- CPU restatement of the reference Qwen3-ASR hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (libqasr.so) never links, loads or calls anything here.
 *
 * It restates, function for function, the reference's CPU path
 * (qwang-sj/qwen3-asr.cpp @ /root/reference) together with the upstream-ggml
 * CPU numerics that path relies on (SURVEY.md §8(a) "ggml numerics" i-ix):
 *   - log-mel front-end           src/mel_spectrogram.cpp:353-415, 484-628
 *   - audio encoder               src/audio_encoder.cpp:12-22, 85-160, 304-601
 *   - text decoder (prefill/step) src/text_decoder.cpp:392-684
 *   - prompt + greedy loop        src/qwen3_asr.cpp:151-317
 *
 * Pinning: the mel stage is pinned bit-for-bit against the reference's own
 * mel_spectrogram.cpp built from /root/reference (oracle/Makefile -> _ref/),
 * see tests/golden/.  The encoder/decoder restatement is pinned only by the
 * reference's structural fixtures (shapes, splice, prompt, tie rule); ggml
 * itself is absent from the reference snapshot (empty submodule), so its
 * floating-point kernels are restated from upstream ggml semantics:
 * "parity partially pinned" (DESIGN.md §Oracle).
 */
#ifndef QASR_ORACLE_H
#define QASR_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QO_N_MEL 128
#define QO_N_FFT 400
#define QO_HOP 160
#define QO_N_BINS 201

/* Weights as host arrays.  2-D weights are IEEE fp16 bit patterns (or raw
 * Q8_0 blocks for the linear weights, see wtype) laid out as
 * in the GGUF file (ggml ne[0] = in_features, i.e. PyTorch [out][in] rows);
 * 1-D tensors are fp32.  Shapes follow src/gguf_loader.cpp:130-190 and
 * src/text_decoder.cpp:175-229. */
typedef struct {
    const uint16_t *attn_q_w, *attn_k_w, *attn_v_w, *attn_out_w;
    const float *attn_q_b, *attn_k_b, *attn_v_b, *attn_out_b;
    const float *attn_norm_w, *attn_norm_b;
    const uint16_t *ffn_up_w, *ffn_down_w;
    const float *ffn_up_b, *ffn_down_b;
    const float *ffn_norm_w, *ffn_norm_b;
} qo_enc_layer;

typedef struct {
    const float *attn_norm, *attn_q_norm, *attn_k_norm, *ffn_norm;
    const uint16_t *attn_q, *attn_k, *attn_v, *attn_output;
    const uint16_t *ffn_gate, *ffn_up, *ffn_down;
} qo_dec_layer;

typedef struct {
    /* audio encoder hparams (src/gguf_loader.h:15-25) */
    int enc_layers, d_model, enc_heads, enc_ffn, conv_ch, n_mel;
    float enc_eps;
    /* text decoder hparams (src/text_decoder.h:15-31) */
    int vocab, hidden, dec_layers, n_head, n_kv_head, head_dim, dec_ffn;
    float rms_eps, rope_theta;
    int eos_id, audio_start_id, audio_end_id, audio_pad_id;
    /* ggml type of the linear 2-D weights (every non-conv matrix except
     * token_embd, scripts/convert_hf_to_gguf.py:230-308): QO_TYPE_F16 or
     * QO_TYPE_Q8_0 (raw block_q8_0 rows, 34 B per 32 values) */
    int wtype;

    const uint16_t *conv1_w, *conv2_w, *conv3_w, *conv_out_w;
    const float *conv1_b, *conv2_b, *conv3_b;
    const float *ln_post_w, *ln_post_b;
    const uint16_t *proj1_w, *proj2_w;
    const float *proj1_b, *proj2_b;
    qo_enc_layer *enc;

    const uint16_t *token_embd;   /* [vocab][hidden] fp16, also the tied LM head */
    const float *output_norm;
    qo_dec_layer *dec;

    /* Qwen3-ForcedAligner (src/forced_aligner.h:36-73): aligner != 0 selects
     * its encoder (chunks zero-padded to 100 frames, 104-frame attention
     * windows, src/forced_aligner.cpp:591-924) and decoder attention (K kept
     * fp32, V cast to fp16, :1041-1046); classify_w = output.weight rows
     * [classify_num][hidden] fp16 (:1073-1076). */
    int aligner, classify_num;
    const uint16_t *classify_w;
} qo_model;

#define QO_TYPE_F16  1
#define QO_TYPE_Q8_0 8

/* numerics switches ("switches for (iii) and (viii)") */
#define QO_GELU_EXACT   1   /* tanh-GELU in fp32 instead of ggml's fp16 LUT   */
#define QO_FA_V_F32     2   /* fp32 V accumulation instead of ggml's fp16 one */
#define QO_FA_V_ROUND1  4   /* fp16 V accumulation, each key's fma rounded once
                               (fp16 of the exact v*vs + acc) instead of ggml's
                               x86 fp32-fma-then-fp16; the scale by ms unchanged */
#define QO_ENC_NO_CHUNK 8   /* AudioEncoder::encode_no_chunk: the conv stack over all
                               frames as one chunk, PE positions 0..N-1 (ASR model) */

/* the V-accumulator step: ggml (F16C) fp16(fmaf(x, v, y)), and the single-
 * rounding variant of QO_FA_V_ROUND1 (fp16 RNE of the exact x * v + y) */
uint16_t qo_f16_mad_round2(uint16_t x, float v, uint16_t y);
uint16_t qo_f16_mad_round1(uint16_t x, float v, uint16_t y);

/* ---------------- fp16 helpers (ggml_compute_fp32_to_fp16, RNE) -------- */
uint16_t qo_f32_to_f16(float f);
float    qo_f16_to_f32(uint16_t h);

/* ---------------- mel front-end ---------------------------------------- */
/* src/mel_spectrogram.cpp:361-415 -> filters[128][201] (mel-major) */
void qo_mel_filters(float *filters);
/* src/mel_spectrogram.cpp:484-628 -> returns n_len, writes out[128][n_len].
 * out may be NULL to query n_len. */
int  qo_log_mel(const float *samples, int n_samples, const float *filters, float *out);
/* src/mel_spectrogram.cpp:130-221 PCM16 RIFF reader; returns n samples or -1.
 * If out is NULL only the count is returned. */
int  qo_load_wav(const char *path, float *out, int max_n, int *sample_rate);

/* ---------------- audio encoder ---------------------------------------- */
/* number of encoder frames for T mel frames (src/audio_encoder.cpp:304-343) */
int  qo_enc_frames(int T);
/* conv front-end + PE only (encode_conv_only analogue): out[N][d_model] */
int  qo_encode_conv(const qo_model *m, const float *mel, int T, float *out, int flags);
/* full encoder: out[N][hidden] */
int  qo_encode(const qo_model *m, const float *mel, int T, float *out, int flags);

/* ---------------- text decoder ----------------------------------------- */
typedef struct qo_dec qo_dec;
qo_dec *qo_dec_new(const qo_model *m, int n_ctx, int flags);
void    qo_dec_free(qo_dec *d);
/* src/text_decoder.cpp:588-684: logits for the LAST row only -> logits[vocab] */
int     qo_dec_forward(qo_dec *d, const int32_t *tokens, int n_tokens,
                       const float *audio, int n_audio, int audio_start_pos,
                       int n_past, float *logits);
/* src/qwen3_asr.cpp:305-317: argmax, strict '>' so the lowest index wins ties */
int32_t qo_argmax(const float *logits, int n);

/* ForcedAligner::forward_decoder (src/forced_aligner.cpp:926-1169): one causal
 * prefill of tokens (positions 0..n-1, audio rows spliced at audio_start_pos),
 * then for each of rows[0..n_rows): output RMSNorm -> classify head ->
 * logits[i][classify_num].  Requires m->aligner. */
int qo_align_forward(const qo_model *m, const int32_t *tokens, int n_tokens, const float *audio, int n_audio,
                     int audio_start_pos, const int *rows, int n_rows, float *logits, int flags);

/* src/qwen3_asr.cpp:151-214 (no system prompt): returns P, ids may be NULL */
int  qo_build_prompt(const qo_model *m, int n_audio, int32_t *ids);

/* Full transcribe_internal without text: PCM -> token ids.
 * max_tokens: decode budget; ignore_eos: fixed-budget throughput mode.
 * Timings (ms) for mel / encode / decode written to t_ms[3] if non-NULL.
 * Returns number of tokens written (trailing EOS popped, as the reference). */
int  qo_transcribe(const qo_model *m, const float *pcm, int n, int max_tokens,
                   int ignore_eos, int flags, int32_t *tokens, double *t_ms);

void qo_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
