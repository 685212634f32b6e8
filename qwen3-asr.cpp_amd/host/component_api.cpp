// component_api.cpp -- the reference's component C++ API over the C-ABI:
//   include/mel_spectrogram.h  (src/mel_spectrogram.h:18-65)
//   include/audio_encoder.h    (src/audio_encoder.h:20-53)
//   include/text_decoder.h     (src/text_decoder.h:107-179)
//   include/audio_injection.h  (src/audio_injection.h:1-110, host helpers)
// The compute (mel, encoder, decoder) runs on the GPU through libqasr.so's
// C entry points; what is here is argument mapping, the reference's error
// strings and the .npy / WAV file helpers.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "audio_encoder.h"
#include "audio_injection.h"
#include "mel_spectrogram.h"
#include "qasr_capi.h"
#include "qasr_host.h"
#include "text_decoder.h"

namespace {

// QASR_DEVICE selects the HIP device of the component objects (default 0)
int component_device() {
    const char *d = getenv("QASR_DEVICE");
    return d ? atoi(d) : 0;
}

// the calling thread's mel engine (created on first use, freed at thread exit)
struct MelEngineHolder {
    qasr_mel_engine *e = nullptr;
    int device = -1;
    ~MelEngineHolder() {
        if (e) qasr_mel_engine_free(e);
    }
};
thread_local MelEngineHolder t_mel;

// numpy .npy header: dtype, shape, fortran order (versions 1.0 and 2.0)
bool read_npy_header(std::ifstream &f, std::vector<size_t> &shape, std::string &dtype, bool &fortran) {
    char magic[6];
    if (!f.read(magic, 6) || memcmp(magic, "\x93NUMPY", 6) != 0) return false;
    unsigned char ver[2];
    if (!f.read((char *)ver, 2)) return false;
    uint32_t hlen = 0;
    if (ver[0] == 1) {
        uint16_t h16 = 0;
        if (!f.read((char *)&h16, 2)) return false;
        hlen = h16;
    } else {
        if (!f.read((char *)&hlen, 4)) return false;
    }
    std::string h(hlen, '\0');
    if (!f.read(&h[0], hlen)) return false;
    auto field = [&](const char *key) -> std::string {
        const size_t k = h.find(key);
        if (k == std::string::npos) return "";
        size_t c = h.find(':', k);
        return c == std::string::npos ? "" : h.substr(c + 1);
    };
    std::string d = field("'descr'");
    const size_t q0 = d.find('\''), q1 = q0 == std::string::npos ? q0 : d.find('\'', q0 + 1);
    if (q1 == std::string::npos) return false;
    dtype = d.substr(q0 + 1, q1 - q0 - 1);
    fortran = field("'fortran_order'").find("True") < field("'fortran_order'").find(',');
    std::string sh = field("'shape'");
    const size_t p0 = sh.find('('), p1 = sh.find(')');
    if (p0 == std::string::npos || p1 == std::string::npos) return false;
    shape.clear();
    std::stringstream ss(sh.substr(p0 + 1, p1 - p0 - 1));
    std::string tok;
    while (std::getline(ss, tok, ','))
        if (tok.find_first_not_of(" ") != std::string::npos) shape.push_back((size_t)std::stoull(tok));
    return true;
}

// float32 / float64 payload of n values into out (as float)
bool read_npy_values(std::ifstream &f, const std::string &dtype, size_t n, float *out) {
    if (dtype == "<f4" || dtype == "float32") return (bool)f.read((char *)out, n * 4);
    if (dtype == "<f8" || dtype == "float64") {
        std::vector<double> d(n);
        if (!f.read((char *)d.data(), n * 8)) return false;
        for (size_t i = 0; i < n; i++) out[i] = (float)d[i];
        return true;
    }
    fprintf(stderr, "Error: Unsupported dtype: %s\n", dtype.c_str());
    return false;
}

}  // namespace

// =================================================================== mel
bool load_wav(const std::string &path, std::vector<float> &samples, int &sample_rate) {
    std::string err;
    if (!qasr::load_wav(path, samples, sample_rate, err)) {
        fprintf(stderr, "Error: %s\n", err.c_str());
        return false;
    }
    return true;
}

bool load_mel_filters_npy(const std::string &path, MelFilters &filters) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) {
        fprintf(stderr, "Error: Cannot open mel filters file: %s\n", path.c_str());
        return false;
    }
    std::vector<size_t> shape;
    std::string dtype;
    bool fortran = false;
    if (!read_npy_header(f, shape, dtype, fortran)) {
        fprintf(stderr, "Error: Invalid NPY header in %s\n", path.c_str());
        return false;
    }
    if (shape.size() != 2) {
        fprintf(stderr, "Error: Expected 2D array for mel filters, got %zu dimensions\n", shape.size());
        return false;
    }
    const size_t nf = shape[0], nm = shape[1];   // file (201, 128) -> filters [128][201]
    std::vector<float> raw(nf * nm);
    if (!read_npy_values(f, dtype, raw.size(), raw.data())) return false;
    filters.n_mel = (int32_t)nm;
    filters.n_fft = (int32_t)nf;
    filters.data.assign(nm * nf, 0.0f);
    for (size_t i = 0; i < nf; i++)
        for (size_t j = 0; j < nm; j++) filters.data[j * nf + i] = raw[i * nm + j];
    return true;
}

void generate_mel_filters(MelFilters &filters, int n_mels, int n_fft, int sample_rate) {
    qasr::mel_filters(filters.data, n_mels, n_fft, sample_rate);
    filters.n_mel = n_mels;
    filters.n_fft = 1 + n_fft / 2;
}

bool log_mel_spectrogram(const float *samples, int n_samples, const MelFilters &filters, MelSpectrogram &mel, int) {
    if (filters.n_mel != QWEN_N_MELS || filters.n_fft != QWEN_N_FFT_BINS ||
        filters.data.size() != (size_t)QWEN_N_MELS * QWEN_N_FFT_BINS) {
        fprintf(stderr, "Error: the GPU mel takes a %d x %d filterbank (got %d x %d)\n", QWEN_N_MELS, QWEN_N_FFT_BINS, filters.n_mel,
                filters.n_fft);
        return false;
    }
    if (n_samples < 0 || (n_samples > 0 && !samples)) return false;
    const int dev = component_device();
    if (!t_mel.e || t_mel.device != dev) {
        if (t_mel.e) qasr_mel_engine_free(t_mel.e);
        t_mel.e = nullptr;
        if (qasr_mel_engine_create(dev, &t_mel.e) != 0) {
            fprintf(stderr, "Error: %s\n", qasr_last_error());
            return false;
        }
        t_mel.device = dev;
    }
    const int T = qasr_mel_frames(n_samples);
    mel.n_mel = QWEN_N_MELS;
    mel.n_len = T;
    mel.n_len_org = T;
    mel.data.assign((size_t)QWEN_N_MELS * T, 0.0f);
    if (qasr_mel_engine_run(t_mel.e, samples, n_samples, filters.data.data(), mel.data.data()) != 0) {
        fprintf(stderr, "Error: %s\n", qasr_last_error());
        return false;
    }
    return true;
}

bool save_mel_npy(const std::string &path, const MelSpectrogram &mel) {
    std::ofstream f(path, std::ios::binary);
    if (!f.is_open()) {
        fprintf(stderr, "Error: Cannot create file: %s\n", path.c_str());
        return false;
    }
    std::string h = "{'descr': '<f4', 'fortran_order': False, 'shape': (" + std::to_string(mel.n_mel) + ", " +
                    std::to_string(mel.n_len) + "), }";
    const size_t total = 10 + h.size() + 1;   // magic + version + length field, header, '\n'
    h.append((64 - total % 64) % 64, ' ');
    h.push_back('\n');
    const uint16_t hl = (uint16_t)h.size();
    f.write("\x93NUMPY\x01\x00", 8);
    f.write((const char *)&hl, 2);
    f.write(h.data(), h.size());
    f.write((const char *)mel.data.data(), mel.data.size() * 4);
    return (bool)f;
}

bool load_mel_npy(const std::string &path, MelSpectrogram &mel) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) {
        fprintf(stderr, "Error: Cannot open file: %s\n", path.c_str());
        return false;
    }
    std::vector<size_t> shape;
    std::string dtype;
    bool fortran = false;
    if (!read_npy_header(f, shape, dtype, fortran)) {
        fprintf(stderr, "Error: Invalid NPY header in %s\n", path.c_str());
        return false;
    }
    if (shape.size() != 2) {
        fprintf(stderr, "Error: Expected 2D array, got %zu dimensions\n", shape.size());
        return false;
    }
    mel.n_mel = (int32_t)shape[0];
    mel.n_len = (int32_t)shape[1];
    mel.n_len_org = mel.n_len;
    mel.data.assign(shape[0] * shape[1], 0.0f);
    return read_npy_values(f, dtype, mel.data.size(), mel.data.data());
}

float compare_mel(const MelSpectrogram &a, const MelSpectrogram &b) {
    if (a.n_mel != b.n_mel || a.n_len != b.n_len) {
        fprintf(stderr, "Error: Mel spectrogram dimensions don't match: (%d, %d) vs (%d, %d)\n", a.n_mel, a.n_len, b.n_mel,
                b.n_len);
        return -1.0f;
    }
    float mx = 0.0f;
    for (size_t i = 0; i < a.data.size(); i++) mx = std::max(mx, std::fabs(a.data[i] - b.data[i]));
    return mx;
}

namespace qwen3_asr {

// =============================================================== encoder
AudioEncoder::AudioEncoder() = default;
AudioEncoder::~AudioEncoder() {
    if (ctx_) qasr_ctx_free(ctx_);
    if (model_) qasr_model_free(model_);
}

bool AudioEncoder::load_model(const std::string &model_path) {
    if (ctx_) { qasr_ctx_free(ctx_); ctx_ = nullptr; }
    if (model_) { qasr_model_free(model_); model_ = nullptr; }
    if (qasr_model_load(model_path.c_str(), component_device(), &model_) != 0) {
        error_msg_ = std::string("Failed to load model: ") + qasr_last_error();
        model_ = nullptr;
        return false;
    }
    qasr_hparams hp;
    qasr_model_hparams(model_, &hp);
    hparams_.n_encoder_layers = hp.enc_layers;
    hparams_.d_model = hp.d_model;
    hparams_.n_attention_heads = hp.enc_heads;
    hparams_.ffn_dim = hp.enc_ffn;
    hparams_.conv_channels = hp.conv_channels;
    hparams_.conv_out_dim = hp.d_model;
    hparams_.n_mel_bins = hp.n_mel;
    hparams_.layer_norm_eps = hp.enc_eps;
    text_hparams_.hidden_size = hp.hidden_size;
    text_hparams_.n_decoder_layers = hp.dec_layers;
    text_hparams_.n_attention_heads = hp.n_heads;
    text_hparams_.n_key_value_heads = hp.n_kv_heads;
    text_hparams_.intermediate_size = hp.dec_ffn;
    text_hparams_.rms_norm_eps = hp.rms_eps;
    // one clip per call; the decoder positions are unused by the encoder
    if (qasr_ctx_create(model_, 1, 64, &ctx_) != 0) {
        error_msg_ = std::string("Failed to create the device context: ") + qasr_last_error();
        ctx_ = nullptr;
        return false;
    }
    return true;
}

bool AudioEncoder::run(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output, bool conv_only) {
    if (!ctx_) {
        error_msg_ = "Model not loaded";
        return false;
    }
    if (!mel_data || n_mel != hparams_.n_mel_bins || n_frames <= 0) {
        error_msg_ = "Expected a [" + std::to_string(hparams_.n_mel_bins) + "][n_frames] mel spectrogram";
        return false;
    }
    const int N = qasr_encoder_frames(n_frames);
    output.assign((size_t)N * (conv_only ? hparams_.d_model : text_hparams_.hidden_size), 0.0f);
    const int rc = conv_only ? qasr_encode_conv(ctx_, mel_data, &n_frames, 1, output.data())
                             : qasr_encode(ctx_, mel_data, &n_frames, 1, output.data());
    if (rc != 0) {
        error_msg_ = std::string("Failed to compute graph: ") + qasr_last_error();
        return false;
    }
    return true;
}

bool AudioEncoder::encode(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output) {
    return run(mel_data, n_mel, n_frames, output, false);
}
bool AudioEncoder::encode_conv_only(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output) {
    return run(mel_data, n_mel, n_frames, output, true);
}
// src/audio_encoder.cpp:603-852: the conv stack over all frames, PE 0..N-1
bool AudioEncoder::encode_no_chunk(const float *mel_data, int n_mel, int n_frames, std::vector<float> &output) {
    if (!ctx_) {
        error_msg_ = "Model not loaded";
        return false;
    }
    if (!mel_data || n_mel != hparams_.n_mel_bins || n_frames <= 0) {
        error_msg_ = "Mel bins mismatch";
        return false;
    }
    output.assign((size_t)qasr_encoder_frames_no_chunk(n_frames) * text_hparams_.hidden_size, 0.0f);
    if (qasr_encode_no_chunk(ctx_, mel_data, &n_frames, 1, output.data()) != 0) {
        error_msg_ = std::string("Failed to compute encoder graph: ") + qasr_last_error();
        return false;
    }
    return true;
}

// =============================================================== decoder
TextDecoder::TextDecoder() = default;
TextDecoder::~TextDecoder() {
    if (ctx_) qasr_ctx_free(ctx_);
    if (model_) qasr_model_free(model_);
}

bool TextDecoder::load_model(const std::string &model_path) {
    if (ctx_) { qasr_ctx_free(ctx_); ctx_ = nullptr; }
    if (model_) { qasr_model_free(model_); model_ = nullptr; }
    n_ctx_ = n_used_ = 0;
    if (qasr_model_load(model_path.c_str(), component_device(), &model_) != 0) {
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
    config_.pad_token_id = hp.pad_id;
    config_.eos_token_id = hp.eos_id;
    config_.audio_start_token_id = hp.audio_start_id;
    config_.audio_end_token_id = hp.audio_end_id;
    config_.audio_pad_token_id = hp.audio_pad_id;
    return true;
}

bool TextDecoder::init_kv_cache(int32_t n_ctx) {
    if (!model_) {
        error_msg_ = "Model not loaded";
        return false;
    }
    if (ctx_) { qasr_ctx_free(ctx_); ctx_ = nullptr; }
    n_ctx_ = n_used_ = 0;
    if (n_ctx <= 0 || qasr_ctx_create(model_, 1, n_ctx, &ctx_) != 0) {
        error_msg_ = std::string("Failed to allocate KV cache buffer: ") + qasr_last_error();
        ctx_ = nullptr;
        return false;
    }
    n_ctx_ = n_ctx;
    return true;
}

void TextDecoder::clear_kv_cache() { n_used_ = 0; }

bool TextDecoder::forward(const int32_t *tokens, int32_t n_tokens, int32_t n_past, std::vector<float> &output) {
    return forward_with_audio(tokens, n_tokens, nullptr, 0, -1, n_past, output);
}

bool TextDecoder::forward_with_audio(const int32_t *tokens, int32_t n_tokens, const float *audio_embd, int32_t n_audio,
                                     int32_t audio_start_pos, int32_t n_past, std::vector<float> &output) {
    if (!model_) {
        error_msg_ = "Model not loaded";
        return false;
    }
    if (n_ctx_ == 0 && !init_kv_cache(1024)) return false;   // src/text_decoder.cpp:600-604
    if (!tokens || n_tokens <= 0 || n_past < 0) {
        error_msg_ = "bad arguments";
        return false;
    }
    if (n_past + n_tokens > n_ctx_) {
        error_msg_ = "Context length exceeded";
        return false;
    }
    // the splice of src/text_decoder.cpp:431: only when the audio rows fit the batch
    const bool splice = audio_embd && n_audio > 0 && audio_start_pos >= 0 && audio_start_pos + n_audio <= n_tokens;
    output.assign((size_t)config_.vocab_size, 0.0f);
    int rc = 0;
    if (n_past == 0) {
        const int P = n_tokens, N = splice ? n_audio : 0, ap = splice ? audio_start_pos : -1;
        rc = qasr_prefill(ctx_, tokens, &P, splice ? audio_embd : nullptr, &ap, &N, 1, output.data(), nullptr);
    } else if (splice) {   // the audio rows of a chunk after cached tokens (src/text_decoder.cpp:588-644)
        const int P = n_tokens, N = n_audio, ap = audio_start_pos;
        rc = qasr_prefill_chunk_audio(ctx_, tokens, &P, &n_past, audio_embd, &ap, &N, 1, output.data(), nullptr);
    } else if (n_tokens == 1) {
        rc = qasr_decode_step(ctx_, tokens, &n_past, 1, output.data(), nullptr);
    } else {
        // one causal chunk prefill over the cache (src/text_decoder.cpp:392-581:
        // one graph for the chunk), the logits of its last row
        const int P = n_tokens;
        rc = qasr_prefill_chunk(ctx_, tokens, &P, &n_past, 1, output.data(), nullptr);
    }
    if (rc != 0) {
        error_msg_ = std::string("Failed to compute graph: ") + qasr_last_error();
        return false;
    }
    n_used_ = n_past + n_tokens;
    return true;
}

std::string TextDecoder::decode_token(int32_t token_id) const { return decode_tokens({token_id}); }

std::string TextDecoder::decode_tokens(const std::vector<int32_t> &tokens) const {
    if (!model_ || tokens.empty()) return "";
    const int n = qasr_detokenize(model_, tokens.data(), (int)tokens.size(), nullptr, 0);
    if (n <= 0) return "";
    std::string s((size_t)n + 1, '\0');
    qasr_detokenize(model_, tokens.data(), (int)tokens.size(), &s[0], n + 1);
    s.resize((size_t)n);
    return s;
}

std::vector<int32_t> TextDecoder::tokenize(const std::string &text) const {
    if (!model_) return {};
    std::vector<int32_t> ids(text.size() * 4 + 16);
    const int n = qasr_tokenize(model_, text.c_str(), ids.data(), (int)ids.size());
    ids.resize(n > 0 ? (size_t)n : 0);
    return ids;
}

// src/text_decoder.cpp:686-760: forward without audio, then the graph tensors
// named debug_norm0, debug_q0_raw, ... -- which the reference's build_graph
// never names (none of them exists in its graph: its map comes back empty) --
// and the logits tensor, which holds the LAST row only (:564-566): the same here
// (the last row's logits; an empty debug map)
bool TextDecoder::forward_debug(const int32_t *tokens, int32_t n_tokens, int32_t n_past, std::vector<float> &output,
                                std::map<std::string, std::vector<float>> &debug_tensors) {
    debug_tensors.clear();
    return forward_with_audio(tokens, n_tokens, nullptr, 0, -1, n_past, output);
}

// ======================================================= audio injection
std::vector<int32_t> find_audio_positions(const int32_t *input_ids, int32_t n_tokens, int32_t audio_pad_token_id) {
    std::vector<int32_t> pos;
    for (int32_t i = 0; i < n_tokens; i++)
        if (input_ids[i] == audio_pad_token_id) pos.push_back(i);
    return pos;
}

void embed_tokens(const int32_t *input_ids, int32_t n_tokens, const float *token_embd, int32_t vocab_size, int32_t hidden_size,
                  float *output) {
    for (int32_t i = 0; i < n_tokens; i++) {
        float *row = output + (size_t)i * hidden_size;
        const int32_t id = input_ids[i];
        if (id >= 0 && id < vocab_size) memcpy(row, token_embd + (size_t)id * hidden_size, (size_t)hidden_size * 4);
        else memset(row, 0, (size_t)hidden_size * 4);
    }
}

bool inject_audio_embeddings(float *token_embeddings, int32_t n_tokens, int32_t hidden_size, const float *audio_features,
                             int32_t n_audio_frames, const std::vector<int32_t> &audio_positions) {
    if ((int32_t)audio_positions.size() != n_audio_frames) return false;
    for (int32_t k = 0; k < n_audio_frames; k++) {
        const int32_t p = audio_positions[k];
        if (p < 0 || p >= n_tokens) return false;
        memcpy(token_embeddings + (size_t)p * hidden_size, audio_features + (size_t)k * hidden_size, (size_t)hidden_size * 4);
    }
    return true;
}

injection_result inject_audio(const int32_t *input_ids, int32_t n_tokens, const float *audio_features, int32_t n_audio_frames,
                              const audio_injection_context &ctx) {
    // src/audio_injection.cpp:74-122: same checks, order and messages
    injection_result r;
    r.seq_len = n_tokens;
    r.hidden_size = ctx.hidden_size;
    if (!ctx.token_embd) {
        r.error_msg = "Token embedding weights not provided";
        return r;
    }
    if (n_tokens <= 0) {
        r.error_msg = "Invalid token count";
        return r;
    }
    const std::vector<int32_t> pos = find_audio_positions(input_ids, n_tokens, ctx.tokens.audio_pad_token_id);
    const bool with_audio = audio_features && n_audio_frames > 0;
    if (with_audio && (int32_t)pos.size() != n_audio_frames) {
        r.error_msg = "Mismatch: " + std::to_string(pos.size()) + " audio_pad tokens but " + std::to_string(n_audio_frames) +
                      " audio frames";
        return r;
    }
    r.embeddings.assign((size_t)n_tokens * ctx.hidden_size, 0.0f);
    embed_tokens(input_ids, n_tokens, ctx.token_embd, ctx.vocab_size, ctx.hidden_size, r.embeddings.data());
    if (with_audio && !pos.empty() &&
        !inject_audio_embeddings(r.embeddings.data(), n_tokens, ctx.hidden_size, audio_features, n_audio_frames, pos)) {
        r.error_msg = "Failed to inject audio embeddings";
        return r;
    }
    r.success = true;
    return r;
}

bool validate_audio_injection(const int32_t *input_ids, int32_t n_tokens, int32_t n_audio_frames, int32_t audio_pad_token_id,
                              std::string &error_msg) {
    const int32_t n = count_audio_pad_tokens(input_ids, n_tokens, audio_pad_token_id);
    if (n != n_audio_frames) {
        error_msg = "Expected " + std::to_string(n_audio_frames) + " audio_pad tokens but found " + std::to_string(n);
        return false;
    }
    return true;
}

int32_t find_audio_start_position(const int32_t *input_ids, int32_t n_tokens, int32_t audio_pad_token_id) {
    for (int32_t i = 0; i < n_tokens; i++)
        if (input_ids[i] == audio_pad_token_id) return i;
    return -1;
}

int32_t count_audio_pad_tokens(const int32_t *input_ids, int32_t n_tokens, int32_t audio_pad_token_id) {
    int32_t n = 0;
    for (int32_t i = 0; i < n_tokens; i++) n += input_ids[i] == audio_pad_token_id;
    return n;
}

}  // namespace qwen3_asr
