// qwen3_asr.cpp -- Qwen3ASR (include/qwen3_asr.h) over the C-ABI.
// Mirrors src/qwen3_asr.cpp:21-327: same error strings, same result fields;
// mel / encode / prefill / greedy decode run on the GPU through qasr_run.
#include "qwen3_asr.h"

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "qasr_host.h"

namespace qwen3_asr {

// per-token callback trampoline (qasr_set_token_callback): the reference calls
// progress_callback(n_generated, max_tokens) after every token and prints every
// 10th (src/qwen3_asr.cpp:255-291); a batch reports its first clip
struct TokenCb {
    const progress_callback_t *cb;
    int max_tokens;
    bool print;
};
static void token_cb(void *user, int seq, int n_generated, int32_t) {
    const TokenCb *t = (const TokenCb *)user;
    if (seq != 0) return;
    if (t->cb && *t->cb) (*t->cb)(n_generated, t->max_tokens);
    if (t->print && n_generated % 10 == 0) fprintf(stderr, "Generated %d tokens...\n", n_generated);
}

// the stream's callback: every clip's tokens (seq = the clip's id), so a
// progress callback sees each clip's running count in turn
static void stream_token_cb(void *user, int seq, int n_generated, int32_t) {
    const TokenCb *t = (const TokenCb *)user;
    if (t->cb && *t->cb) (*t->cb)(n_generated, t->max_tokens);
    if (t->print && n_generated % 10 == 0) fprintf(stderr, "Clip %d: generated %d tokens...\n", seq, n_generated);
}

static int64_t now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Qwen3ASR::Qwen3ASR() = default;

Qwen3ASR::~Qwen3ASR() {
    if (ctx_) qasr_ctx_free(ctx_);
    if (model_) qasr_model_free(model_);
}

bool Qwen3ASR::load_model(const std::string &model_path) {
    const int64_t t0 = now_ms();
    if (model_) { qasr_model_free(model_); model_ = nullptr; }
    if (qasr_model_load(model_path.c_str(), device_, &model_) != 0) {
        error_msg_ = std::string("Failed to load model: ") + qasr_last_error();
        model_ = nullptr;
        return false;
    }
    qasr_hparams hp;
    qasr_model_hparams(model_, &hp);
    config_.vocab_size = hp.vocab_size;
    config_.hidden_size = hp.hidden_size;
    config_.n_decoder_layers = hp.dec_layers;
    config_.n_attention_heads = hp.n_heads;
    config_.n_key_value_heads = hp.n_kv_heads;
    config_.intermediate_size = hp.dec_ffn;
    config_.head_dim = hp.head_dim;
    config_.rms_norm_eps = hp.rms_eps;
    config_.rope_theta = hp.rope_theta;
    config_.eos_token_id = hp.eos_id;
    config_.audio_start_token_id = hp.audio_start_id;
    config_.audio_end_token_id = hp.audio_end_id;
    config_.audio_pad_token_id = hp.audio_pad_id;
    fprintf(stderr, "Model loaded in %lld ms\n", (long long)(now_ms() - t0));
    return true;
}

// The shape a context is recreated with when (batch, n_ctx) does not fit the
// current (cur_b, cur_l): the union of both only while its KV cells (slots x
// positions) are no more than the larger of the two shapes' own -- a long
// single clip after a many-slot stream gets (1, its length), not (slots, its
// length), which multiplies the cache (128 slots x 16k positions of
// a 20-min file is ~240 GB of KV at 0.6B).
extern "C" void qasr_ctx_grow_shape(int cur_b, int cur_l, int batch, int n_ctx, int *nb, int *nl) {
    const long long cur = (long long)cur_b * cur_l, want = (long long)batch * n_ctx;
    const int ub = std::max(batch, cur_b), ul = std::max(n_ctx, cur_l);
    if ((long long)ub * ul <= std::max(cur, want)) { *nb = ub; *nl = ul; }
    else { *nb = batch; *nl = n_ctx; }
}

bool Qwen3ASR::ensure_ctx(int batch, int n_ctx) {
    if (ctx_ && ctx_batch_ >= batch && ctx_len_ >= n_ctx) return true;
    if (ctx_) { qasr_ctx_free(ctx_); ctx_ = nullptr; }
    int nb = 0, nl = 0;
    qasr_ctx_grow_shape(ctx_batch_, ctx_len_, batch, n_ctx, &nb, &nl);
    if (qasr_ctx_create(model_, nb, nl, &ctx_) != 0) {
        error_msg_ = std::string("Failed to initialize KV cache: ") + qasr_last_error();
        ctx_ = nullptr;
        return false;
    }
    ctx_batch_ = nb;
    ctx_len_ = nl;
    return true;
}

transcribe_result Qwen3ASR::transcribe(const std::string &audio_path, const transcribe_params &params) {
    transcribe_result result;
    if (!model_) { result.error_msg = "Model not loaded"; return result; }
    std::vector<float> samples;
    int sr = 0;
    if (!load_audio_file(audio_path, samples, sr)) {
        result.error_msg = "Failed to load audio file: " + audio_path;
        return result;
    }
    if (sr != 16000) {
        result.error_msg = "Audio must be 16kHz, got " + std::to_string(sr) + " Hz";
        return result;
    }
    return transcribe_internal(samples.data(), (int)samples.size(), params);
}

transcribe_result Qwen3ASR::transcribe(const float *samples, int n_samples, const transcribe_params &params) {
    transcribe_result result;
    if (!model_) { result.error_msg = "Model not loaded"; return result; }
    return transcribe_internal(samples, n_samples, params);
}

// one clip through qasr_run: the stage timings and --profile sections of the
// reference's transcribe_internal (src/qwen3_asr.cpp:81-160)
std::vector<transcribe_result> Qwen3ASR::transcribe_run(const std::vector<std::vector<float>> &clips,
                                                        const transcribe_params &params) {
    const int B = (int)clips.size();
    std::vector<transcribe_result> out(B);
    if (!model_) { for (auto &r : out) r.error_msg = "Model not loaded"; return out; }
    int maxP = 0;
    std::vector<const float *> ptr(B);
    std::vector<int> n(B);
    for (int b = 0; b < B; b++) {
        ptr[b] = clips[b].data();
        n[b] = (int)clips[b].size();
        maxP = std::max(maxP, qasr_prompt_len(qasr_encoder_frames(qasr_mel_frames(n[b]))));
    }
    const int64_t t0 = now_ms();
    std::vector<int32_t> sys;
    if (!params.system_prompt.empty()) {
        const int k = qasr_tokenize(model_, params.system_prompt.c_str(), nullptr, 0);
        sys.resize(std::max(k, 0));
        qasr_tokenize(model_, params.system_prompt.c_str(), sys.data(), k);
    }
    if (!ensure_ctx(B, maxP + (int)sys.size() + params.max_tokens)) {
        for (auto &r : out) r.error_msg = error_msg_;
        return out;
    }
    qasr_set_system_prompt(ctx_, sys.data(), (int)sys.size());
    qasr_set_profile(ctx_, profile_ ? 1 : 0);   // resets the sections: the report covers this call
    std::vector<int32_t> toks((size_t)B * params.max_tokens);
    std::vector<int> nt(B);
    qasr_timings tm{};
    TokenCb tcb{&progress_callback_, params.max_tokens, params.print_progress};
    const bool per_token = progress_callback_ || params.print_progress;
    qasr_set_token_callback(ctx_, per_token ? token_cb : nullptr, per_token ? &tcb : nullptr);
    const int rc = qasr_transcribe_batch(ctx_, ptr.data(), n.data(), B, params.max_tokens, 0, toks.data(), nt.data(), &tm);
    qasr_set_token_callback(ctx_, nullptr, nullptr);
    if (rc != 0) {
        for (auto &r : out) r.error_msg = std::string("Decoding failed: ") + qasr_last_error();
        return out;
    }
    if (profile_) {
        const int len = qasr_profile_report(ctx_, nullptr, 0);
        std::string rep(std::max(len, 0) + 1, '\0');
        qasr_profile_report(ctx_, &rep[0], (int)rep.size());
        rep.resize(std::max(len, 0));
        profile_report_ = rep;
    }
    const int64_t t1 = now_ms();
    for (int b = 0; b < B; b++) {
        transcribe_result &r = out[b];
        r.tokens.assign(toks.begin() + (long)b * params.max_tokens, toks.begin() + (long)b * params.max_tokens + nt[b]);
        const int len = qasr_detokenize(model_, r.tokens.data(), (int)r.tokens.size(), nullptr, 0);
        std::string text(std::max(len, 0) + 1, '\0');
        qasr_detokenize(model_, r.tokens.data(), (int)r.tokens.size(), &text[0], (int)text.size());
        text.resize(std::max(len, 0));
        r.text = text;
        r.success = true;
        r.t_mel_ms = (int64_t)tm.t_mel_ms;
        r.t_encode_ms = (int64_t)tm.t_encode_ms;
        r.t_decode_ms = (int64_t)(tm.t_prefill_ms + tm.t_decode_ms);
        r.t_total_ms = t1 - t0;
    }
    return out;
}

// several clips: the continuous-batching stream (qasr_run_stream), up to
// max_batch() slots; each clip succeeds or fails on its own, with the
// reference's per-call error strings
std::vector<transcribe_result> Qwen3ASR::transcribe_batch(const std::vector<std::vector<float>> &clips,
                                                          const transcribe_params &params) {
    if (clips.size() <= 1) return transcribe_run(clips, params);
    if (!model_) return std::vector<transcribe_result>(clips.size(), [] { transcribe_result r; r.error_msg = "Model not loaded"; return r; }());
    std::vector<transcribe_result> out(clips.size());
    int maxP = 0;
    for (const auto &c : clips) maxP = std::max(maxP, qasr_prompt_len(qasr_encoder_frames(qasr_mel_frames((int)c.size()))));
    const int n_sys = params.system_prompt.empty() ? 0 : std::max(qasr_tokenize(model_, params.system_prompt.c_str(), nullptr, 0), 0);
    size_t next = 0;
    const bool ok = transcribe_stream(
        [&](int &id, std::vector<float> &pcm) {
            if (next >= clips.size()) return false;
            id = (int)next;
            pcm = clips[next++];
            return true;
        },
        [&](int id, transcribe_result r) { out[id] = std::move(r); }, params, maxP + n_sys + params.max_tokens,
        std::min((int)clips.size(), max_batch_));
    if (!ok)
        for (auto &r : out)
            if (!r.success && r.error_msg.empty()) r.error_msg = error_msg_;
    return out;
}

namespace {
struct StreamCtx {
    const std::function<bool(int &, std::vector<float> &)> *fetch;
    const std::function<void(int, transcribe_result)> *sink;
    qasr_model *model;
    std::vector<float> pcm;
    int64_t t0;
};
int stream_fetch(void *u, const float **pcm, int *n, int *) {
    StreamCtx *s = (StreamCtx *)u;
    int id = -1;
    if (!(*s->fetch)(id, s->pcm) || id < 0) return -1;
    *pcm = s->pcm.data();
    *n = (int)s->pcm.size();
    return id;
}
void stream_sink(void *u, int id, int status, const int32_t *toks, int n) {
    StreamCtx *s = (StreamCtx *)u;
    transcribe_result r;
    if (status != 0) {
        r.error_msg = std::string("Decoding failed: ") + qasr_last_error();
    } else {
        r.tokens.assign(toks, toks + n);
        const int len = qasr_detokenize(s->model, toks, n, nullptr, 0);
        std::string text(std::max(len, 0) + 1, '\0');
        qasr_detokenize(s->model, toks, n, &text[0], (int)text.size());
        text.resize(std::max(len, 0));
        r.text = text;
        r.success = true;
        r.t_total_ms = now_ms() - s->t0;   // (completion time within the stream)
    }
    (*s->sink)(id, std::move(r));
}
}  // namespace

bool Qwen3ASR::transcribe_stream(const std::function<bool(int &id, std::vector<float> &pcm)> &fetch,
                                 const std::function<void(int id, transcribe_result result)> &sink,
                                 const transcribe_params &params, int n_ctx, int slots) {
    if (!model_) { error_msg_ = "Model not loaded"; return false; }
    std::vector<int32_t> sys;
    if (!params.system_prompt.empty()) {
        const int k = qasr_tokenize(model_, params.system_prompt.c_str(), nullptr, 0);
        sys.resize(std::max(k, 0));
        qasr_tokenize(model_, params.system_prompt.c_str(), sys.data(), k);
    }
    // context length: n_ctx, or the prompt of a 30 s clip (the reference's
    // chunking unit) plus the budget -- longer clips fail alone ("Context length")
    const int need = n_ctx > 0 ? n_ctx : qasr_prompt_len(qasr_encoder_frames(qasr_mel_frames(30 * 16000))) + (int)sys.size() + params.max_tokens;
    const int S = slots > 0 ? std::min(slots, max_batch_) : max_batch_;
    if (!ensure_ctx(S, need)) return false;
    qasr_set_system_prompt(ctx_, sys.data(), (int)sys.size());
    qasr_set_profile(ctx_, profile_ ? 1 : 0);   // the report covers the whole stream
    TokenCb tcb{&progress_callback_, params.max_tokens, params.print_progress};
    const bool per_token = progress_callback_ || params.print_progress;
    qasr_set_token_callback(ctx_, per_token ? stream_token_cb : nullptr, per_token ? &tcb : nullptr);
    StreamCtx sc{&fetch, &sink, model_, {}, now_ms()};
    const int rc = qasr_run_stream(ctx_, S, stream_fetch, stream_sink, &sc, params.max_tokens, 0, nullptr);
    qasr_set_token_callback(ctx_, nullptr, nullptr);
    if (rc != 0) { error_msg_ = std::string("Decoding failed: ") + qasr_last_error(); return false; }
    if (profile_) {
        const int len = qasr_profile_report(ctx_, nullptr, 0);
        std::string rep(std::max(len, 0) + 1, '\0');
        qasr_profile_report(ctx_, &rep[0], (int)rep.size());
        rep.resize(std::max(len, 0));
        profile_report_ = rep;
    }
    return true;
}

transcribe_result Qwen3ASR::transcribe_internal(const float *samples, int n_samples, const transcribe_params &params) {
    std::vector<std::vector<float>> one(1, std::vector<float>(samples, samples + n_samples));
    transcribe_result r = transcribe_run(one, params)[0];
    if (r.success && params.print_timing) {
        fprintf(stderr, "\nTiming:\n");
        fprintf(stderr, "  Mel spectrogram: %lld ms\n", (long long)r.t_mel_ms);
        fprintf(stderr, "  Audio encoding:  %lld ms\n", (long long)r.t_encode_ms);
        fprintf(stderr, "  Text decoding:   %lld ms\n", (long long)r.t_decode_ms);
        fprintf(stderr, "  Total:           %lld ms\n", (long long)r.t_total_ms);
        fprintf(stderr, "  Tokens generated: %zu\n", r.tokens.size());
    }
    return r;
}

void Qwen3ASR::set_progress_callback(progress_callback_t callback) { progress_callback_ = std::move(callback); }

bool load_audio_file(const std::string &path, std::vector<float> &samples, int &sample_rate) {
    std::string err;
    if (!qasr::load_wav(path, samples, sample_rate, err)) {
        fprintf(stderr, "Error: %s\n", err.c_str());
        return false;
    }
    return true;
}

}  // namespace qwen3_asr
