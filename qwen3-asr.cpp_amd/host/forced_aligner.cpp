// forced_aligner.cpp -- ForcedAligner (include/forced_aligner.h) over the C-ABI.
// Mirrors src/forced_aligner.cpp:57-134 (load_model), :1564-1720 (tokenize /
// align): same error strings and result fields; mel, encoder, prefill and the
// classification head run on the GPU through qasr_align, the LIS repair and
// the class -> seconds conversion on the host exactly as the reference.
#include "forced_aligner.h"

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "qwen3_asr.h"

namespace qwen3_asr {

static int64_t now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

ForcedAligner::ForcedAligner() = default;

ForcedAligner::~ForcedAligner() {
    if (ctx_) qasr_ctx_free(ctx_);
    if (model_) qasr_model_free(model_);
}

bool ForcedAligner::load_model(const std::string &model_path) {
    if (ctx_) { qasr_ctx_free(ctx_); ctx_ = nullptr; ctx_len_ = 0; }
    if (model_) { qasr_model_free(model_); model_ = nullptr; }
    if (qasr_model_load(model_path.c_str(), device_, &model_) != 0) {
        error_msg_ = std::string("Failed to open GGUF file: ") + model_path + " (" + qasr_last_error() + ")";
        model_ = nullptr;
        return false;
    }
    qasr_hparams hp;
    qasr_model_hparams(model_, &hp);
    if (hp.classify_num <= 0) {
        error_msg_ = "Not a ForcedAligner model (no classification head): " + model_path;
        qasr_model_free(model_);
        model_ = nullptr;
        return false;
    }
    hparams_.audio_encoder_layers = hp.enc_layers;
    hparams_.audio_d_model = hp.d_model;
    hparams_.audio_attention_heads = hp.enc_heads;
    hparams_.audio_ffn_dim = hp.enc_ffn;
    hparams_.text_decoder_layers = hp.dec_layers;
    hparams_.text_hidden_size = hp.hidden_size;
    hparams_.vocab_size = hp.vocab_size;
    hparams_.classify_num = hp.classify_num;
    hparams_.timestamp_token_id = hp.timestamp_token_id;
    return true;
}

bool ForcedAligner::ensure_ctx(int n_ctx) {
    if (ctx_ && ctx_len_ >= n_ctx) return true;
    if (ctx_) { qasr_ctx_free(ctx_); ctx_ = nullptr; }
    const int nl = std::max(n_ctx, ctx_len_);
    if (qasr_ctx_create(model_, 1, nl, &ctx_) != 0) {
        error_msg_ = std::string("Failed to allocate KV cache buffer: ") + qasr_last_error();
        ctx_ = nullptr;
        return false;
    }
    ctx_len_ = nl;
    return true;
}

bool ForcedAligner::load_korean_dict(const std::string &dict_path) {
    if (!model_ || qasr_model_load_korean_dict(model_, dict_path.c_str()) != 0) return false;
    fprintf(stderr, "Korean dictionary loaded: %s\n", dict_path.c_str());
    return true;
}

std::vector<int32_t> ForcedAligner::tokenize_with_timestamps(const std::string &text, std::vector<std::string> &words,
                                                             const std::string &language) {
    words.clear();
    if (!model_) return {};
    const int wl = qasr_align_words(model_, text.c_str(), language.c_str(), nullptr, 0);
    std::string joined(std::max(wl, 0) + 1, '\0');
    qasr_align_words(model_, text.c_str(), language.c_str(), &joined[0], (int)joined.size());
    joined.resize(std::max(wl, 0));
    for (size_t st = 0; !joined.empty() && st <= joined.size();) {
        const size_t e = joined.find('\n', st);
        words.push_back(joined.substr(st, e == std::string::npos ? std::string::npos : e - st));
        if (e == std::string::npos) break;
        st = e + 1;
    }
    int nw = 0;
    const int n = qasr_align_tokenize(model_, text.c_str(), language.c_str(), nullptr, 0, &nw);
    std::vector<int32_t> ids(std::max(n, 0));
    qasr_align_tokenize(model_, text.c_str(), language.c_str(), ids.data(), n, &nw);
    return ids;
}

alignment_result ForcedAligner::align(const std::string &audio_path, const std::string &text, const std::string &language) {
    alignment_result result;
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
    return align(samples.data(), (int)samples.size(), text, language);
}

alignment_result ForcedAligner::align(const float *samples, int n_samples, const std::string &text,
                                      const std::string &language) {
    alignment_result result;
    const int64_t t0 = now_ms();
    if (!model_) { result.error_msg = "Model not loaded"; return result; }
    if (n_samples <= 0) { result.error_msg = "Failed to compute mel spectrogram"; return result; }
    const float audio_duration = (float)n_samples / 16000.0f;
    std::vector<std::string> words;
    const std::vector<int32_t> ids = tokenize_with_timestamps(text, words, language);
    if (!ensure_ctx(qasr_align_prompt_len(n_samples, (int)ids.size()))) { result.error_msg = error_msg_; return result; }
    std::vector<int32_t> cls(std::max<size_t>(ids.size(), 1));
    int nts = 0;
    qasr_timings tm{};
    if (qasr_align(ctx_, samples, n_samples, ids.data(), (int)ids.size(), cls.data(), (int)cls.size(), &nts, &tm) != 0) {
        result.error_msg = std::string("Decoder forward pass failed: ") + qasr_last_error();
        return result;
    }
    cls.resize(nts);
    std::vector<int32_t> fixed(nts);
    if (nts) qasr_fix_timestamps(cls.data(), nts, fixed.data());
    // classes_to_timestamps + clamp (src/forced_aligner.cpp:1267-1278, 1694-1714)
    const float seg = hparams_.timestamp_segment_time_ms / 1000.0f;
    std::vector<float> ts(nts);
    for (int i = 0; i < nts; i++) ts[i] = std::min(fixed[i] * seg, audio_duration);
    for (size_t i = 0; i < words.size(); i++) {
        aligned_word aw;
        aw.word = words[i];
        aw.start = 2 * i < ts.size() ? ts[2 * i] : 0.0f;
        aw.end = 2 * i + 1 < ts.size() ? ts[2 * i + 1] : audio_duration;
        result.words.push_back(aw);
    }
    result.t_mel_ms = (int64_t)tm.t_mel_ms;
    result.t_encode_ms = (int64_t)tm.t_encode_ms;
    result.t_decode_ms = (int64_t)tm.t_prefill_ms;
    result.success = true;
    result.t_total_ms = now_ms() - t0;
    return result;
}

}  // namespace qwen3_asr
