// forced_aligner.h -- C++17 ForcedAligner API of the reference
// (src/forced_aligner.h:15-33 aligned_word / alignment_result,
// :199-282 class ForcedAligner), implemented over the C-ABI of libqasr.so
// (include/qasr_capi.h: qasr_align*, qasr_model_load_korean_dict) instead of
// ggml graphs.  Model files: Qwen3-ForcedAligner GGUF (classification head
// output.weight, 24 x 1024 audio encoder).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "qasr_capi.h"

namespace qwen3_asr {

// src/forced_aligner.h:15-33
struct aligned_word {
    std::string word;
    float start;   // seconds
    float end;     // seconds
};

struct alignment_result {
    std::vector<aligned_word> words;
    bool success = false;
    std::string error_msg;
    int64_t t_mel_ms = 0;
    int64_t t_encode_ms = 0;
    int64_t t_decode_ms = 0;
    int64_t t_total_ms = 0;
};

// src/forced_aligner.h:36-73 (the values a loaded model reports)
struct forced_aligner_hparams {
    int32_t audio_encoder_layers = 24;
    int32_t audio_d_model = 1024;
    int32_t audio_attention_heads = 16;
    int32_t audio_ffn_dim = 4096;
    int32_t text_decoder_layers = 28;
    int32_t text_hidden_size = 1024;
    int32_t vocab_size = 152064;
    int32_t classify_num = 5000;
    int32_t timestamp_token_id = 151705;
    int32_t timestamp_segment_time_ms = 80;
};

// src/forced_aligner.h:199-282
class ForcedAligner {
public:
    ForcedAligner();
    ~ForcedAligner();
    ForcedAligner(const ForcedAligner &) = delete;
    ForcedAligner &operator=(const ForcedAligner &) = delete;

    bool load_model(const std::string &model_path);
    alignment_result align(const std::string &audio_path, const std::string &text, const std::string &language = "");
    alignment_result align(const float *samples, int n_samples, const std::string &text, const std::string &language = "");
    const std::string &get_error() const { return error_msg_; }
    bool is_loaded() const { return model_ != nullptr; }
    const forced_aligner_hparams &get_hparams() const { return hparams_; }
    std::vector<int32_t> tokenize_with_timestamps(const std::string &text, std::vector<std::string> &words,
                                                  const std::string &language = "");
    bool load_korean_dict(const std::string &dict_path);

    // MI355X addition: device selection
    void set_device(int device) { device_ = device; }

private:
    bool ensure_ctx(int n_ctx);

    qasr_model *model_ = nullptr;
    qasr_ctx *ctx_ = nullptr;
    int ctx_len_ = 0, device_ = 0;
    forced_aligner_hparams hparams_;
    std::string error_msg_;
};

}  // namespace qwen3_asr
