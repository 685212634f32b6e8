// audio_encoder.h -- the reference's AudioEncoder component
// (src/audio_encoder.h:20-53, hparams src/gguf_loader.h:15-35), implemented
// by libqasr.so over the C-ABI (qasr_encode / qasr_encode_conv): the conv
// front-end and the 18-layer encoder run as the MI355X kernels of csrc/ on the
// device selected by QASR_DEVICE (default 0).  No ggml types: the weights
// live in the device arena of a qasr_model.  A reference caller (e.g.
// tests/test_encoder.cpp) recompiles against this header unchanged.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "qasr_capi.h"

namespace qwen3_asr {

// src/gguf_loader.h:15-25
struct audio_encoder_hparams {
    int32_t n_encoder_layers = 18;
    int32_t d_model = 896;
    int32_t n_attention_heads = 14;
    int32_t ffn_dim = 3584;
    int32_t conv_channels = 480;
    int32_t conv_out_dim = 896;
    int32_t n_mel_bins = 128;
    int32_t n_window_infer = 800;
    float layer_norm_eps = 1e-5f;
};

// src/gguf_loader.h:28-35
struct text_decoder_hparams {
    int32_t hidden_size = 1024;
    int32_t n_decoder_layers = 28;
    int32_t n_attention_heads = 16;
    int32_t n_key_value_heads = 8;
    int32_t intermediate_size = 3072;
    float rms_norm_eps = 1e-6f;
};

class AudioEncoder {
public:
    AudioEncoder();
    ~AudioEncoder();
    AudioEncoder(const AudioEncoder &) = delete;
    AudioEncoder &operator=(const AudioEncoder &) = delete;

    // src/audio_encoder.cpp:42-83
    bool load_model(const std::string &model_path);

    // mel_data: [n_mel][n_frames] mel-major; output: [N][hidden_size] with
    // N = qasr_encoder_frames(n_frames) (src/audio_encoder.cpp:312-601)
    bool encode(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output);

    // the conv front-end + positional embedding only: [N][d_model]
    bool encode_conv_only(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output);

    // the reference's un-chunked debug path (src/audio_encoder.cpp:603-737):
    // not provided -- the encoder here always runs the reference's 100-frame
    // chunking; returns false with an error message
    bool encode_no_chunk(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output);

    const audio_encoder_hparams &get_hparams() const { return hparams_; }
    const text_decoder_hparams &get_text_hparams() const { return text_hparams_; }
    const std::string &get_error() const { return error_msg_; }

private:
    bool run(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output, bool conv_only);

    qasr_model *model_ = nullptr;
    qasr_ctx *ctx_ = nullptr;
    audio_encoder_hparams hparams_;
    text_decoder_hparams text_hparams_;
    std::string error_msg_;
};

}  // namespace qwen3_asr
