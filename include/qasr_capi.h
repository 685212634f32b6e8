/*
 * qasr_capi.h -- C-ABI of the MI355X-native Qwen3-ASR engine (libqasr.so).
 *
 * The reference has no plugin registry; its hot-path boundary is the C++
 * class API listed below.  Each entry point here replaces one of those calls
 * (SURVEY.md §8(b)); plain pointers and sizes only, no torch / HIP types.
 *
 *   qasr_model_load / qasr_model_free
 *       <- Qwen3ASR::load_model           src/qwen3_asr.cpp:21-42
 *          (AudioEncoder::load_model      src/audio_encoder.cpp:42-83,
 *           TextDecoder::load_model       src/text_decoder.cpp:38-114,
 *           GGUFLoader::load              src/gguf_loader.cpp:17-53)
 *   qasr_ctx_create / qasr_ctx_free
 *       <- TextDecoder::init_kv_cache     src/text_decoder.cpp:337-386
 *   qasr_mel, qasr_mel_engine_run
 *       <- log_mel_spectrogram            src/mel_spectrogram.h:53-55 / .cpp:484-628
 *   qasr_mel_filters
 *       <- generate_mel_filters           src/mel_spectrogram.h:42-43 / .cpp:352-395
 *   qasr_encode, qasr_encode_conv
 *       <- AudioEncoder::encode           src/audio_encoder.h:27 / .cpp:312-601
 *          AudioEncoder::encode_conv_only src/audio_encoder.h:30
 *   qasr_prefill
 *       <- TextDecoder::forward_with_audio src/text_decoder.h:134-137 / .cpp:588-684
 *   qasr_decode_step
 *       <- TextDecoder::forward           src/text_decoder.h:125-126 / .cpp:583-586
 *          + Qwen3ASR::sample_greedy      src/qwen3_asr.cpp:305-317 (fused argmax)
 *   qasr_transcribe_batch / qasr_stage_audio + qasr_run
 *       <- Qwen3ASR::transcribe_internal  src/qwen3_asr.cpp:81-149
 *          + decode_greedy                src/qwen3_asr.cpp:216-303
 *   qasr_detokenize / qasr_tokenize
 *       <- TextDecoder::decode_tokens / tokenize src/text_decoder.cpp:1069-1103
 *   qasr_align, qasr_align_json          (ForcedAligner model files)
 *       <- ForcedAligner::align           src/forced_aligner.cpp:1636-1720
 *          (encode_audio :591-924, forward_decoder :1088-1169,
 *           extract_timestamp_classes :1280-1306)
 *   qasr_align_tokenize <- ForcedAligner::tokenize_with_timestamps :1564-1609
 *   qasr_model_load_korean_dict <- ForcedAligner::load_korean_dict :1543-1562
 *   qasr_fix_timestamps <- ForcedAligner::fix_timestamp_classes :1183-1265
 *
 * Conventions (mirroring the reference's):
 *   - return value: 0 = OK, nonzero = error; message via qasr_last_error().
 *     Nothing throws across the boundary.
 *   - host pointers are caller-owned; outputs are written into caller
 *     buffers sized by the documented formula (query helpers provided).
 *   - a context owns its device buffers, KV cache and HIP stream; calls on
 *     one context are stream-ordered and NOT thread-safe (one context per
 *     host thread), exactly as the reference's objects.
 *   - layouts: mel [128][T] mel-major; features [N][1024] row-major; logits
 *     [151936] fp32 (last row only); token ids int32.
 */
#ifndef QASR_CAPI_H
#define QASR_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qasr_model qasr_model;
typedef struct qasr_ctx qasr_ctx;

#define QASR_OK 0
#define QASR_ERR_ARG 1
#define QASR_ERR_IO 2
#define QASR_ERR_FORMAT 3
#define QASR_ERR_DEVICE 4
#define QASR_ERR_STATE 5

typedef struct {
    /* audio encoder (src/gguf_loader.h:15-25) */
    int32_t enc_layers, d_model, enc_heads, enc_ffn, conv_channels, n_mel;
    float enc_eps;
    /* text decoder (src/text_decoder.h:15-31) */
    int32_t vocab_size, hidden_size, dec_layers, n_heads, n_kv_heads, head_dim, dec_ffn;
    float rms_eps, rope_theta;
    int32_t eos_id, pad_id, audio_start_id, audio_end_id, audio_pad_id;
    int32_t weight_type; /* ggml type of the 2-D linear weights: 1 = F16, 8 = Q8_0 */
    /* Qwen3-ForcedAligner files (src/forced_aligner.h:36-73): classify_num > 0 */
    int32_t classify_num, timestamp_token_id;
} qasr_hparams;

typedef struct {
    double t_mel_ms, t_encode_ms, t_prefill_ms, t_decode_ms, t_total_ms;  /* device (HIP event) time */
    int32_t n_decode_steps;
} qasr_timings;

/* ---- errors / version ---------------------------------------------------- */
const char *qasr_last_error(void);                 /* thread-local last message */
const char *qasr_version(void);
int qasr_device_count(int *n);
/* Self-check of the exact prefill attention's expf (fa_exact.hip px_expf_nonpos,
 * the device expf's instruction sequence without its overflow clamp) against the
 * device expf on every non-positive fp32 input (2^31 + 1 values) on `device`:
 * *mismatches = the number of differing results (0 = the kernel's weights are
 * ggml's expf bits).  No reference counterpart (a property of this build). */
int qasr_check_expf_nonpos(int device, uint64_t *mismatches);

/* ---- model ---------------------------------------------------------------- */
/* device >= 0: upload weights to that HIP device.  device = QASR_HOST_ONLY:
 * parse + validate the GGUF and load the tokenizer only (no GPU needed);
 * such a model serves hparams/text calls but cannot create a context. */
#define QASR_HOST_ONLY (-1)
int qasr_model_load(const char *gguf_path, int device, qasr_model **out);
void qasr_model_free(qasr_model *m);
int qasr_model_hparams(const qasr_model *m, qasr_hparams *out);
/* device bytes held by the weight arena */
int64_t qasr_model_device_bytes(const qasr_model *m);

/* ---- context -------------------------------------------------------------- */
/* max_batch: clips per call; max_ctx: decoder positions per sequence
 * (prompt + max_tokens, src/qwen3_asr.cpp:223). */
int qasr_ctx_create(qasr_model *m, int max_batch, int max_ctx, qasr_ctx **out);
void qasr_ctx_free(qasr_ctx *c);

/* ---- size helpers (host-only arithmetic) ---------------------------------- */
int qasr_mel_frames(int n_samples);               /* n/160 (src/mel_spectrogram.cpp:517-522) */
int qasr_encoder_frames(int n_mel_frames);        /* src/audio_encoder.cpp:304-343 */
int qasr_prompt_len(int n_audio_frames);          /* n + 15 (src/qwen3_asr.cpp:170-209) */
/* build the reference chat prompt (no system prompt); returns P, writes
 * ids[P] and the first <|audio_pad|> index to *audio_pos. */
int qasr_build_prompt(const qasr_model *m, int n_audio_frames, int32_t *ids, int *audio_pos);

/* ---- stages (host buffers in/out; each call synchronises its stream) ---- */
/* B clips: pcm[b] has n[b] samples; mel_out receives B blocks of [128][T_b]
 * back to back, T_b = qasr_mel_frames(n[b]). */
int qasr_mel(qasr_ctx *c, const float *const *pcm, const int *n, int B, float *mel_out);
/* mel: B blocks [128][T_b] back to back; feats: [sum N_b][hidden] */
int qasr_encode(qasr_ctx *c, const float *mel, const int *T, int B, float *feats);
/* conv front-end + positional embedding only: [sum N_b][d_model] */
int qasr_encode_conv(qasr_ctx *c, const float *mel, const int *T, int B, float *out);
/* AudioEncoder::encode_no_chunk (src/audio_encoder.cpp:603-852): the conv stack
 * over each clip's T_b frames as ONE chunk (no 100-frame split), sinusoidal PE
 * positions 0 .. N_b - 1, then the same transformer; feats [sum N_b][hidden]
 * with N_b = qasr_encoder_frames_no_chunk(T_b).  ASR models only. */
int qasr_encode_no_chunk(qasr_ctx *c, const float *mel, const int *T, int B, float *feats);
int qasr_encoder_frames_no_chunk(int n_mel_frames);
/* Prefill B sequences from n_past = 0 (the KV cache of sequence b is reset).
 * ids: sum P_b tokens back to back; feats: sum N_b rows of [hidden];
 * audio_pos[b]: first pad index (splice rows [audio_pos, audio_pos+N_b));
 * logits_last (optional) [B][vocab]; argmax (optional) [B]. */
int qasr_prefill(qasr_ctx *c, const int32_t *ids, const int *P, const float *feats,
                 const int *audio_pos, const int *N, int B, float *logits_last, int32_t *argmax);
/* A chunk of P[b] tokens after n_past[b] cached ones (no audio splice), one
 * causal prefill over the cache and the chunk; logits of each chunk's last
 * row.  <- TextDecoder::forward(tokens, n_tokens > 1, n_past > 0)
 *    src/text_decoder.h:125-126 / .cpp:392-581, 583-586 */
int qasr_prefill_chunk(qasr_ctx *c, const int32_t *ids, const int *P, const int *n_past, int B,
                       float *logits_last, int32_t *argmax);
/* The same chunk with audio rows spliced in (feats: sum N_b rows of [hidden];
 * rows [audio_pos[b], audio_pos[b] + N_b) of chunk b when they fit in it).
 * <- TextDecoder::forward_with_audio(tokens, n, audio, n_audio, pos, n_past)
 *    at any n_past, src/text_decoder.cpp:588-644 (splice :431-459) */
int qasr_prefill_chunk_audio(qasr_ctx *c, const int32_t *ids, const int *P, const int *n_past, const float *feats,
                             const int *audio_pos, const int *N, int B, float *logits_last, int32_t *argmax);
/* One decode step for B sequences at positions n_past[b] (token tok[b]). */
int qasr_decode_step(qasr_ctx *c, const int32_t *tok, const int *n_past, int B,
                     float *logits, int32_t *argmax);

/* ---- standalone log-mel (no model) ----------------------------------------- */
/* log_mel_spectrogram of src/mel_spectrogram.h:53-55 without a model: an
 * engine keeps the DFT / window tables and a filterbank on one device and runs
 * the context's mel kernels.  filters: [128][201] (NULL: the built-in
 * generate_mel_filters values); mel_out: [128][qasr_mel_frames(n)].  One
 * engine per host thread. */
typedef struct qasr_mel_engine qasr_mel_engine;
int qasr_mel_engine_create(int device, qasr_mel_engine **out);
void qasr_mel_engine_free(qasr_mel_engine *e);
int qasr_mel_engine_run(qasr_mel_engine *e, const float *pcm, int n, const float *filters, float *mel_out);
/* host: generate_mel_filters(128, 400, 16000) (src/mel_spectrogram.cpp:352-395) -> out[128][201] */
int qasr_mel_filters(float *out);

/* ---- whole path ----------------------------------------------------------- */
/* Stage PCM into device HBM (one H2D copy); qasr_run then works from HBM.
 * Any number of clips may be staged (a pool); qasr_run needs B <= max_batch,
 * qasr_run_staged runs subsets of a larger pool. */
int qasr_stage_audio(qasr_ctx *c, const float *const *pcm, const int *n, int B);
/* Greedy transcription of staged clips clips[0..B) (indices into the last
 * qasr_stage_audio call, B <= max_batch) as one batch, from HBM; outputs as
 * qasr_run.  The multi-GPU sharded driver stages a rank's whole shard once
 * and runs it batch by batch (bench.py --utterances). */
int qasr_run_staged(qasr_ctx *c, const int *clips, int B, int max_tokens, int ignore_eos, int32_t *tokens,
                    int *n_tokens, qasr_timings *t);
/* Greedy transcription of the staged clips: tokens [B][max_tokens],
 * n_tokens[B] (trailing EOS popped as src/qwen3_asr.cpp:298-300).
 * ignore_eos != 0: fixed budget of max_tokens steps (throughput mode). */
int qasr_run(qasr_ctx *c, int max_tokens, int ignore_eos, int32_t *tokens, int *n_tokens,
             qasr_timings *t);
/* Optional system-prompt token ids inserted by qasr_run after
 * "<|im_start|>system\n" (src/qwen3_asr.cpp:186-190); n = 0 clears. */
int qasr_set_system_prompt(qasr_ctx *c, const int32_t *ids, int n);
int qasr_transcribe_batch(qasr_ctx *c, const float *const *pcm, const int *n, int B, int max_tokens,
                          int ignore_eos, int32_t *tokens, int *n_tokens, qasr_timings *t);

/* ---- continuous batching ---------------------------------------------------- */
/* Greedy transcription of a queue of clips through `slots` KV-cache slots
 * (1..max_batch; 0 = max_batch) decoding as one batch: a slot whose clip ends (EOS unless ignore_eos, or its token
 * budget) is refilled from the queue at the next chunk boundary (<= 8 decode
 * steps; 1 with a token callback), so a batch never waits for its longest
 * member.  Clip results equal qasr_run's for the same clip.
 *   fetch(user, &pcm, &n_samples, &max_tokens): the next clip -> its id
 *       (>= 0), 16 kHz mono samples (read before fetch is called again) and
 *       its budget (preset to the call's max_tokens); < 0: the queue is empty
 *       (fetch is not called again).  A shared counter behind fetch makes a
 *       dynamic work queue across contexts, threads or processes.
 *   sink(user, id, status, tokens, n_tokens): once per fetched clip, in
 *       completion order: status 0 with the tokens (trailing EOS popped, as
 *       qasr_run), or a QASR_ERR_* code for that clip alone (no audio frames,
 *       context length exceeded, bad arguments) with qasr_last_error() set
 *       during the call; the run goes on with the other clips.
 * The token callback (qasr_set_token_callback) receives the clip id as seq.
 * Returns non-zero only for failures of the run itself (device errors). */
typedef int (*qasr_fetch_fn)(void *user, const float **pcm, int *n_samples, int *max_tokens);
typedef void (*qasr_sink_fn)(void *user, int id, int status, const int32_t *tokens, int n_tokens);
typedef struct {
    int32_t n_clips, n_errors, n_prefills;  /* clips delivered, clips rejected, refill prefills */
    int64_t n_steps;                        /* decode steps (each over all the slots) */
    int64_t slot_steps, live_steps;         /* slot-steps run, of which decoding a live clip */
    double t_prefill_ms, t_decode_ms, t_total_ms;  /* host wall time: refills, decode chunks, call */
    double t_mel_ms, t_encode_ms;           /* device time (HIP events) of the refills' mel / encoder stages,
                                               parts of t_prefill_ms */
    int64_t kv_keys;                        /* sum over decode steps and slots of the keys each slot's attention
                                               read (n_kv): the steps' K / V cache bytes = kv_keys x layers x
                                               n_kv_heads x 128 x 2 B x 2 */
} qasr_stream_stats;
int qasr_run_stream(qasr_ctx *c, int slots, qasr_fetch_fn fetch, qasr_sink_fn sink, void *user, int max_tokens, int ignore_eos,
                    qasr_stream_stats *stats);
/* The same over the staged pool (qasr_stage_audio; inputs already in HBM):
 * fetch(user, &max_tokens) returns the next clip's id (>= 0), or < 0 when the
 * queue is empty; the clip is staged clip id.  An id outside the pool fails
 * that clip (QASR_ERR_ARG through the sink) unless the context option
 * "staged_wrap" is 1: then it is staged clip id % (pool size), so an utterance
 * set larger than the pool reuses its clips, each under its own id. */
typedef int (*qasr_fetch_staged_fn)(void *user, int *max_tokens);
int qasr_run_stream_staged(qasr_ctx *c, int slots, qasr_fetch_staged_fn fetch, qasr_sink_fn sink, void *user,
                           int max_tokens, int ignore_eos, qasr_stream_stats *stats);

/* ---- per-context options (no reference counterpart: MI355X launch tuning) -- */
/* Batch-1 decode runs two fused launches per layer whose roles wait on each
 * other in-launch.  Options, defaulted from the environment
 * variable in brackets at qasr_ctx_create:
 *   "fuse_ffn" [QASR_FUSE_FFN], "fuse_qkv" [QASR_FUSE_QKV], "fuse_o" [QASR_FUSE_O]
 *       1/0: the fused launch or the separate launches (same arithmetic)
 *   "ffn_delay", "ffn_wdelay", "qkv_delay", "o_delay"  in-launch delays (~0.2 us units)
 *   "att_spl1" [QASR_ATT_SPL1]   batch <= 8 attention key split: 0 auto, 64, 128
 *   "poll_limit" [QASR_POLL_LIMIT]  bounded in-launch waits (polls); a wait that
 *       runs out makes the call fail with QASR_ERR_DEVICE
 *   "handoff_fence" [QASR_HANDOFF_FENCE]  1: agent-scope release/acquire fences
 *       around every in-launch hand-off (diagnostic)
 *   "dec_layers"  diagnostic: decode steps run only the first n decoder layers (0 = all)
 * Read-only: "slots_ffn", "slots_qkv" (co-resident workgroups of the fused
 * kernels on the context's device).  Setting an option drops captured decode
 * graphs.  Unknown names: QASR_ERR_ARG. */
int qasr_ctx_set_option(qasr_ctx *c, const char *name, int value);
int qasr_ctx_get_option(const qasr_ctx *c, const char *name, int *value);
/* diagnostic copy of decode-step state (after qasr_decode_step): "x" fp32
 * [max_batch][hidden] residual stream, "act" fp16 [max_batch][ffn] SwiGLU
 * output, "qkv" fp32 [max_batch][q+k+v], "att" fp16 [max_batch][n_head*128] */
int qasr_debug_read(qasr_ctx *c, const char *buffer, void *dst, int64_t bytes);

/* Per-token callback (Qwen3ASR::set_progress_callback, src/qwen3_asr.cpp:255-291):
 * called synchronously on the caller's thread after every greedy token of
 * qasr_run / qasr_run_staged -- the prefill's token first (n_generated = 1) --
 * for every sequence still decoding, in sequence order.  Each step then
 * synchronises the stream (the token must reach the host), so a callback
 * costs throughput; NULL removes it.  The callback must not start another
 * qasr_run / qasr_run_staged / qasr_run_stream* / qasr_decode_step on any
 * context of the same GPU: a batch-1 run holds that device's fused-launch
 * lock (not recursive) while it calls back. */
int qasr_set_token_callback(qasr_ctx *c, void (*cb)(void *user, int seq, int n_generated, int32_t token), void *user);

/* ---- measurement ---------------------------------------------------------- */
/* --profile (src/timing.h QWEN3_TIMER sections, src/main.cpp:409-411): on = 1
 * records per-section device time (HIP events) of every qasr_run --
 * mel_spectrogram, audio_encoding.{total,conv_chunk,transformer},
 * decode.initial_forward, decode.token (one per step), transcribe.total --
 * accumulated until the next qasr_set_profile (which resets).  The run also
 * carries roctx ranges "qasr.run" / "qasr.decode" for rocprofv3 --marker-trace. */
int qasr_set_profile(qasr_ctx *c, int on);
/* the report in QWEN3_TIMER_REPORT's layout; returns its length, writes at
 * most cap-1 bytes + NUL */
int qasr_profile_report(qasr_ctx *c, char *out, int cap);
/* Probe one launch group of every greedy decode step of qasr_run with HIP
 * events on the context's stream: kernel 1 = LM head + fused argmax; 2 = the
 * QKV projection + attention (+ o-projection) of decoder layer "probe_layer"
 * (option, default 14) -- at batch 1 the fused qkv_attn1_kernel; 3 = that
 * layer's FFN (batch 1: ffn1_kernel).  The rest of each step replays as two
 * graphs around it (one extra graph launch per step); 0 disables.  Setting a
 * probe resets the totals; bytes_per_launch = mean algorithmic HBM bytes of
 * the probed launches (weights + the layer's K/V rows at each step's n_kv).
 * 4 = at decode batches (9..128 rows) that layer's attention launch alone
 * (decode_attn_seq_kernel: K / V^T rows + q / output rows), by the device
 * clock (qasr_get_probe_device). */
int qasr_set_probe(qasr_ctx *c, int kernel);
int qasr_get_probe(qasr_ctx *c, double *total_ms, int64_t *launches, double *bytes_per_launch);
/* The same launches timed by the device clock (first workgroup start -> last
 * workgroup end, 100 MHz s_memrealtime, folded in-kernel by the batch <= 8
 * decode kernels and the decode-batch attention): the kernels' own duration, without the ~2.5 us of dispatch
 * and event processing an event pair around one launch includes. */
int qasr_get_probe_device(qasr_ctx *c, double *total_ms, int64_t *launches);

/* ---- forced alignment (Qwen3-ForcedAligner model files) ------------------- */
/* Device part of ForcedAligner::align for one clip: text_ids are the words'
 * BPE ids, each word followed by two timestamp tokens (qasr_align_tokenize);
 * classes[i] = argmax class of the i-th timestamp token (x 80 ms), *n_ts =
 * their number (writes at most cap).  The context needs max_ctx >=
 * qasr_align_prompt_len.  t: t_mel_ms, t_encode_ms, t_prefill_ms (= decode). */
int qasr_align(qasr_ctx *c, const float *pcm, int n_samples, const int32_t *text_ids, int n_text,
               int32_t *classes, int cap, int *n_ts, qasr_timings *t);
/* words -> ids with timestamps; language "korean" uses the loaded dictionary
 * (qasr_model_load_korean_dict), else whitespace words.  Returns the number of
 * ids (writes at most cap); *n_words = number of words. */
int qasr_align_tokenize(const qasr_model *m, const char *text, const char *language, int32_t *ids, int cap,
                        int *n_words);
/* the words of that split, joined by '\n' (words never contain whitespace);
 * returns the length, writes at most cap-1 bytes + NUL */
int qasr_align_words(const qasr_model *m, const char *text, const char *language, char *out, int cap);
int qasr_model_load_korean_dict(qasr_model *m, const char *path);
/* Host policy of the Qwen3ASR class (no reference counterpart): the shape a
 * context (cur_b slots x cur_l positions) is recreated with for a call that
 * needs (batch, n_ctx) -- the union of both while its KV cells do not exceed
 * the larger shape's own, else exactly (batch, n_ctx). */
void qasr_ctx_grow_shape(int cur_b, int cur_l, int batch, int n_ctx, int *nb, int *nl);
/* LIS repair of raw classes (in -> out, n values) */
int qasr_fix_timestamps(const int32_t *classes, int n, int32_t *out);
/* prompt length of an alignment: n_text + 2 + pads(mel frames of n_samples) */
int qasr_align_prompt_len(int n_samples, int n_text);
/* The whole alignment -> the CLI's JSON document {"words": [{"word", "start",
 * "end"}...]} (src/main.cpp:257-276).  Returns its length (or minus the error
 * code on failure); writes at most cap-1 bytes + NUL. */
int qasr_align_json(qasr_ctx *c, const float *pcm, int n_samples, const char *text, const char *language,
                    char *out, int cap, qasr_timings *t);
/* B clips in one aligner pass (mel + windowed encoder of all clips, one
 * prefill of the B prompts, one classify GEMM over every timestamp row): the
 * B documents of qasr_align_json as one JSON array, in input order; each
 * clip's classes equal its single-clip run.  B <= the context's max_batch.
 * Returns the length (or minus the error code); writes at most cap-1 + NUL.
 * <- the --transcribe-align pipeline over many files, src/main.cpp:416-500 */
int qasr_align_json_batch(qasr_ctx *c, const float *const *pcm, const int *n_samples, const char *const *text, int B,
                          const char *language, char *out, int cap, qasr_timings *t);

/* ---- text (host) ---------------------------------------------------------- */
/* UTF-8 text for ids (special <|..|> and [PAD..] tokens skipped); returns the
 * byte length (excluding NUL), writes at most cap-1 bytes + NUL. */
int qasr_detokenize(const qasr_model *m, const int32_t *ids, int n, char *out, int cap);
/* byte-level BPE; returns number of ids (writes at most cap). */
int qasr_tokenize(const qasr_model *m, const char *text, int32_t *ids, int cap);

/* ---- host utilities (no device needed) ------------------------------------ */
/* PCM16 RIFF reader (src/mel_spectrogram.cpp:130-221); returns n or -1.
 * out may be NULL to query n. */
int qasr_load_wav(const char *path, float *out, int max_n, int *sample_rate);
int qasr_write_wav(const char *path, const float *pcm, int n, int sample_rate);
/* deterministic synthetic clip: seed 1000+i recipe */
int qasr_synth_pcm(uint64_t seed, int n_samples, float *out);
/* synthetic GGUF with the reference tensor names/shapes/dtypes.
 * config: "full" (Qwen3-ASR-0.6B dims) or "tiny" (test dims);
 * wtype: 1 = f16, 8 = q8_0 for linear weights. */
int qasr_write_synthetic_gguf(const char *path, const char *config, uint64_t seed, int wtype);
/* version of that writer's output: bumped whenever the file it writes for a
 * given (config, seed, wtype) changes, so a cached synthetic model is keyed on it */
int qasr_synthetic_gguf_version(void);

#ifdef __cplusplus
}
#endif
#endif
