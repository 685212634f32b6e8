// ref_shim.cpp -- extern "C" entry points over the REFERENCE's own sources.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile together with
// /root/reference/src/mel_spectrogram.cpp and src/audio_injection.cpp (left
// where they lie, never copied) into oracle/_ref/libqasr_ref.so.  Used to pin
// the oracle restatement and to generate tests/golden/ fixtures.  These are
// the only reference translation units that build without ggml
// (SURVEY.md §8(c)); everything else in the reference needs the absent ggml.
#include "mel_spectrogram.h"
#include "audio_injection.h"

#include <cstring>
#include <vector>

extern "C" {

// src/mel_spectrogram.cpp:361-415
void ref_mel_filters(float *out) {
    MelFilters f;
    generate_mel_filters(f, QWEN_N_MELS, QWEN_N_FFT, QWEN_SAMPLE_RATE);
    std::memcpy(out, f.data.data(), f.data.size() * sizeof(float));
}

// src/mel_spectrogram.cpp:484-628; returns n_len, out may be NULL (query).
int ref_log_mel(const float *samples, int n, float *out) {
    MelFilters f;
    generate_mel_filters(f, QWEN_N_MELS, QWEN_N_FFT, QWEN_SAMPLE_RATE);
    MelSpectrogram mel;
    if (!log_mel_spectrogram(samples, n, f, mel, 1)) return -1;
    if (out) std::memcpy(out, mel.data.data(), mel.data.size() * sizeof(float));
    return mel.n_len;
}

// src/mel_spectrogram.cpp:130-221
int ref_load_wav(const char *path, float *out, int max_n, int *sample_rate) {
    std::vector<float> s;
    int sr = 0;
    if (!load_wav(path, s, sr)) return -1;
    if (sample_rate) *sample_rate = sr;
    if (out) {
        int n = (int)s.size() < max_n ? (int)s.size() : max_n;
        std::memcpy(out, s.data(), n * sizeof(float));
    }
    return (int)s.size();
}

// src/audio_injection.cpp: embed_tokens + inject_audio_embeddings
int ref_inject_audio(const int32_t *ids, int n_tokens, const float *audio, int n_audio,
                     const float *token_embd, int vocab, int hidden, int32_t pad_id, float *out) {
    qwen3_asr::audio_injection_context ctx;
    ctx.token_embd = token_embd;
    ctx.vocab_size = vocab;
    ctx.hidden_size = hidden;
    ctx.tokens.audio_pad_token_id = pad_id;
    auto r = qwen3_asr::inject_audio(ids, n_tokens, audio, n_audio, ctx);
    if (!r.success) return -1;
    std::memcpy(out, r.embeddings.data(), r.embeddings.size() * sizeof(float));
    return r.seq_len;
}

}  // extern "C"
