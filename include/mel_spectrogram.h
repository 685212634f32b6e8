// mel_spectrogram.h -- the reference's log-mel component API
// (src/mel_spectrogram.h:1-67), implemented by libqasr.so: log_mel_spectrogram
// runs the MI355X mel kernels (csrc/mel.hip, through qasr_mel_engine_* of
// include/qasr_capi.h) on the calling thread's device (QASR_DEVICE, default
// 0); the file helpers (WAV, .npy) are host code.  A reference caller
// recompiles against this header unchanged.
#ifndef MEL_SPECTROGRAM_H
#define MEL_SPECTROGRAM_H

#include <cstdint>
#include <string>
#include <vector>

// src/mel_spectrogram.h:8-15
constexpr int QWEN_SAMPLE_RATE = 16000;
constexpr int QWEN_N_FFT = 400;
constexpr int QWEN_HOP_LENGTH = 160;
constexpr int QWEN_N_MELS = 128;
constexpr int QWEN_CHUNK_SIZE = 30;                                   // seconds
constexpr int QWEN_N_SAMPLES = QWEN_SAMPLE_RATE * QWEN_CHUNK_SIZE;    // 480000
constexpr int QWEN_N_FFT_BINS = 1 + (QWEN_N_FFT / 2);                 // 201

// src/mel_spectrogram.h:18-23: [n_mel][n_len], mel-major
struct MelSpectrogram {
    int32_t n_mel;
    int32_t n_len;
    int32_t n_len_org;
    std::vector<float> data;
};

// src/mel_spectrogram.h:26-30: [n_mel][n_fft] (n_fft = 201 bins)
struct MelFilters {
    int32_t n_mel;
    int32_t n_fft;
    std::vector<float> data;
};

// 16-bit PCM mono WAV -> samples in [-1, 1] (src/mel_spectrogram.cpp:130-221)
bool load_wav(const std::string &path, std::vector<float> &samples, int &sample_rate);

// (201, 128) float32/float64 .npy -> filters [128][201] (src/mel_spectrogram.cpp:292-349)
bool load_mel_filters_npy(const std::string &path, MelFilters &filters);

// Slaney-normalised HTK-scale filterbank (src/mel_spectrogram.cpp:352-395)
void generate_mel_filters(MelFilters &filters, int n_mels = QWEN_N_MELS, int n_fft = QWEN_N_FFT,
                          int sample_rate = QWEN_SAMPLE_RATE);

// log10 mel power, clamped to max - 8, (x + 4) / 4; the last STFT frame
// dropped (src/mel_spectrogram.cpp:484-628).  On the GPU: filters must be
// 128 x 201 (any values); n_threads is accepted and unused.
bool log_mel_spectrogram(const float *samples, int n_samples, const MelFilters &filters, MelSpectrogram &mel,
                         int n_threads = 1);

// .npy (float32, shape (n_mel, n_len)) round trip and comparison
// (src/mel_spectrogram.cpp:631-727)
bool save_mel_npy(const std::string &path, const MelSpectrogram &mel);
bool load_mel_npy(const std::string &path, MelSpectrogram &mel);
float compare_mel(const MelSpectrogram &a, const MelSpectrogram &b);

#endif  // MEL_SPECTROGRAM_H
