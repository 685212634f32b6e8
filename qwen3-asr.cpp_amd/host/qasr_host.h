// qasr_host.h -- host-side pieces of the engine (no device code):
// hyper-parameters + tensor contract, precomputed tables, WAV I/O, BPE text.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "gguf.h"

namespace qasr {

struct Hparams {
    // audio encoder: src/gguf_loader.h:15-25 (+ text hidden :28-35)
    int enc_layers = 18, d_model = 896, enc_heads = 14, enc_ffn = 3584, conv_ch = 480, n_mel = 128;
    float enc_eps = 1e-5f;
    // text decoder: src/text_decoder.cpp:116-147
    int vocab = 151936, hidden = 1024, dec_layers = 28, n_head = 16, n_kv_head = 8, head_dim = 128, dec_ffn = 3072;
    float rms_eps = 1e-6f, rope_theta = 1000000.0f;
    int eos_id = 151645, pad_id = 151643, audio_start_id = 151669, audio_end_id = 151670, audio_pad_id = 151676;
    int weight_type = 1;
    // ForcedAligner files (src/forced_aligner.h:36-73; keys convert_hf_to_gguf.py:454-458):
    // classification head output.weight [hidden][classify_num], no chat template
    bool aligner = false;
    int classify_num = 0, timestamp_id = 151705, ts_segment_ms = 80;
};

// Reads hparams with the reference's keys and defaults.  Encoder keys: the
// reference's own (src/gguf_loader.cpp:69-85) first, then the converter's
// (scripts/convert_hf_to_gguf.py:442-447) -- for any converted Qwen3-ASR-0.6B
// file both resolve to the reference's hard-coded defaults.
Hparams read_hparams(const GGUFFile &f);

// ---- precomputed tables (computed on the host exactly as the reference) ----
// src/mel_spectrogram.cpp:361-415
void mel_filters(std::vector<float> &f /*[n_mels][1 + n_fft/2]*/, int n_mels = 128, int n_fft = 400, int sr = 16000);
// src/audio_encoder.cpp:12-22 (positions 0..n_ctx-1)
void sinusoidal_pe(std::vector<float> &pe, int n_ctx, int d_model);
// ggml_table_gelu_f16 (ggml tanh-GELU fp16 table)
void gelu_table(std::vector<uint16_t> &t /*65536*/);
// ggml_rope_cache_init (NEOX, ext_factor 0): [n_pos][head_dim/2] (cos, sin)
void rope_table(std::vector<float> &cs /*[n_pos][hd/2][2]*/, int n_pos, int head_dim, float base);
// DFT twiddles exactly as the reference's fp64 loop evaluates them
// (angle = 2.0*M_PI*k*n/400): [n=400][k=201] (cos, sin)
void dft_twiddles(std::vector<double> &tw /*[400][201][2]*/);
void hann_window(std::vector<double> &w /*400*/);

uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);

// ---- audio ----
bool load_wav(const std::string &path, std::vector<float> &samples, int &sample_rate, std::string &err);
bool write_wav(const std::string &path, const float *pcm, int n, int sample_rate);
void synth_pcm(uint64_t seed, int n, float *out);
int mel_frames(int n_samples);
int encoder_frames(int T);
int chunk_out_len(int L);

// ---- text: byte-level BPE (src/text_decoder.cpp:799-1103) ----
class Tokenizer {
public:
    bool load(const GGUFFile &f, std::string &err);
    std::string decode(const std::vector<int32_t> &ids) const;
    std::string decode_token(int32_t id) const;
    std::vector<int32_t> encode(const std::string &text) const;
    // one word, no leading-space marker; unknown subwords are skipped with a
    // warning (src/forced_aligner.cpp:1589-1603)
    std::vector<int32_t> encode_word(const std::string &word) const;
    size_t size() const { return vocab_.size(); }

private:
    std::vector<std::string> vocab_;
    std::unordered_map<std::string, int32_t> tok2id_;
    std::unordered_map<std::string, int> ranks_;
};

// ---- prompt: src/qwen3_asr.cpp:151-214 ----
std::vector<int32_t> build_prompt(const Hparams &hp, int n_audio, const std::vector<int32_t> &sys_ids, int *audio_pos);

// ---- forced aligner host logic (src/forced_aligner.cpp) ----
// whitespace words (' ', '\t', '\n', '\r'), :1577-1586
std::vector<std::string> split_words(const std::string &text);
// LTokenizer-style Korean split with the jieba word list, :1485-1541
std::vector<std::string> tokenize_korean(const std::string &text, const std::unordered_map<std::string, int> &dict);
bool load_korean_dict(const std::string &path, std::unordered_map<std::string, int> &dict);
// HF _get_feat_extract_output_lengths: number of <|audio_pad|> tokens, :1173-1178
int feat_extract_output_lengths(int mel_frames);
// LIS-based timestamp repair (HF fix_timestamp), :1183-1265
std::vector<int32_t> fix_timestamp_classes(const std::vector<int32_t> &data);
// <|audio_start|> pad x n <|audio_end|> text..., :1308-1329; audio starts at index 1
std::vector<int32_t> build_align_tokens(const Hparams &hp, const std::vector<int32_t> &text_tokens, int n_pads);

// ---- synthetic model ----
bool write_synthetic_gguf(const std::string &path, const std::string &config, uint64_t seed, int wtype, std::string &err);

}  // namespace qasr
