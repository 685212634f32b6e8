// text_decoder.h -- the reference's TextDecoder component
// (src/text_decoder.h:15-31 config, :107-179 class), implemented by libqasr.so
// over the C-ABI: a KV cache is a qasr_ctx (max_batch 1, max_ctx = n_ctx) on
// the device selected by QASR_DEVICE (default 0); forward_with_audio at
// n_past = 0 is qasr_prefill (one causal prefill, audio rows spliced at
// audio_start_pos), a one-token forward at n_past > 0 is qasr_decode_step (the
// batch-1 fused launches), a longer one at n_past > 0 runs the tokens as
// decode steps in order.  As the reference's graph (src/text_decoder.cpp:
// 562-575: a view of the last row before the output norm), `output` holds
// the LAST row's logits only: [vocab_size].  No ggml types; a reference
// caller (tests/test_decoder_simple.cpp, test_decoder_last_pos.cpp,
// test_decoder_no_audio.cpp) recompiles against this header unchanged.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "qasr_capi.h"

namespace qwen3_asr {

// src/text_decoder.h:15-31 (filled from the GGUF by load_model)
struct text_decoder_config {
    int32_t vocab_size = 151936;
    int32_t hidden_size = 1024;
    int32_t n_decoder_layers = 28;
    int32_t n_attention_heads = 16;
    int32_t n_key_value_heads = 8;
    int32_t intermediate_size = 3072;
    int32_t head_dim = 128;
    float rms_norm_eps = 1e-6f;
    float rope_theta = 1000000.0f;
    int32_t pad_token_id = 151643;
    int32_t eos_token_id = 151645;
    int32_t audio_start_token_id = 151669;
    int32_t audio_end_token_id = 151670;
    int32_t audio_pad_token_id = 151676;
};

class TextDecoder {
public:
    TextDecoder();
    ~TextDecoder();
    TextDecoder(const TextDecoder &) = delete;
    TextDecoder &operator=(const TextDecoder &) = delete;

    // src/text_decoder.cpp:38-114
    bool load_model(const std::string &model_path);
    // src/text_decoder.cpp:337-386: a fresh cache of n_ctx positions
    bool init_kv_cache(int32_t n_ctx);
    // src/text_decoder.cpp:388-390
    void clear_kv_cache();

    // src/text_decoder.cpp:583-586
    bool forward(const int32_t *tokens, int32_t n_tokens, int32_t n_past, std::vector<float> &output);
    // src/text_decoder.cpp:588-684: audio_embd [n_audio][hidden_size] replaces
    // the embeddings of tokens [audio_start_pos, audio_start_pos + n_audio)
    // (src/text_decoder.cpp:431-459); splicing needs n_past = 0
    bool forward_with_audio(const int32_t *tokens, int32_t n_tokens, const float *audio_embd, int32_t n_audio,
                            int32_t audio_start_pos, int32_t n_past, std::vector<float> &output);

    const text_decoder_config &get_config() const { return config_; }
    const std::string &get_error() const { return error_msg_; }

    // src/text_decoder.cpp:985-1103
    std::string decode_token(int32_t token_id) const;
    std::string decode_tokens(const std::vector<int32_t> &tokens) const;
    std::vector<int32_t> tokenize(const std::string &text) const;

    // the reference's intermediate-tensor dump (src/text_decoder.cpp:686-
    // 983, ggml graph names): not provided -- intermediate state is read with
    // qasr_debug_read; returns false with an error message
    bool forward_debug(const int32_t *tokens, int32_t n_tokens, int32_t n_past, std::vector<float> &output,
                       std::map<std::string, std::vector<float>> &debug_tensors);

    // MI355X additions: the underlying C-ABI objects (null before load /
    // init_kv_cache) for callers that mix both layers
    qasr_model *c_model() const { return model_; }
    qasr_ctx *c_ctx() const { return ctx_; }

private:
    qasr_model *model_ = nullptr;
    qasr_ctx *ctx_ = nullptr;
    int32_t n_ctx_ = 0, n_used_ = 0;
    text_decoder_config config_;
    std::string error_msg_;
};

}  // namespace qwen3_asr
