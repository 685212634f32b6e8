// audio_injection.h -- the reference's host-side audio injection helpers
// (src/audio_injection.h:1-110), implemented by libqasr.so on host arrays.
// The engine's own splice never materialises embeddings on the host: the
// decoder's embedding-gather kernel (csrc/elementwise.hip launch_embed)
// reads audio rows in place of the <|audio_pad|> rows during the prefill;
// these helpers serve callers of the reference's API that build the combined
// embedding table themselves.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace qwen3_asr {

struct audio_token_ids {
    int32_t audio_start_token_id = 151669;
    int32_t audio_end_token_id = 151670;
    int32_t audio_pad_token_id = 151676;
};

struct injection_result {
    std::vector<float> embeddings;   // [seq_len][hidden_size]
    int32_t seq_len = 0;
    int32_t hidden_size = 0;
    bool success = false;
    std::string error_msg;
};

struct audio_injection_context {
    const float *token_embd = nullptr;   // [vocab_size][hidden_size]
    int32_t vocab_size = 0;
    int32_t hidden_size = 0;
    audio_token_ids tokens;
};

// positions i with input_ids[i] == audio_pad_token_id, in order
std::vector<int32_t> find_audio_positions(const int32_t *input_ids, int32_t n_tokens, int32_t audio_pad_token_id);
// output[i] = token_embd[input_ids[i]] (out-of-range ids: zero rows)
void embed_tokens(const int32_t *input_ids, int32_t n_tokens, const float *token_embd, int32_t vocab_size, int32_t hidden_size,
                  float *output);
// token_embeddings[audio_positions[k]] = audio_features[k] (masked_scatter);
// false when the counts differ or a position is out of range
bool inject_audio_embeddings(float *token_embeddings, int32_t n_tokens, int32_t hidden_size, const float *audio_features,
                             int32_t n_audio_frames, const std::vector<int32_t> &audio_positions);
// embed + inject
injection_result inject_audio(const int32_t *input_ids, int32_t n_tokens, const float *audio_features, int32_t n_audio_frames,
                              const audio_injection_context &ctx);
// the number of <|audio_pad|> tokens equals n_audio_frames
bool validate_audio_injection(const int32_t *input_ids, int32_t n_tokens, int32_t n_audio_frames, int32_t audio_pad_token_id,
                              std::string &error_msg);
// first <|audio_pad|> index, or -1
int32_t find_audio_start_position(const int32_t *input_ids, int32_t n_tokens, int32_t audio_pad_token_id);
int32_t count_audio_pad_tokens(const int32_t *input_ids, int32_t n_tokens, int32_t audio_pad_token_id);

}  // namespace qwen3_asr
