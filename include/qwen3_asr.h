// qwen3_asr.h -- C++17 pipeline API, kept verbatim from the reference's
// src/qwen3_asr.h:15-116 (transcribe_params / transcribe_result / Qwen3ASR),
// implemented over the C-ABI of libqasr.so (include/qasr_capi.h) instead of
// ggml graphs.  Existing callers of the reference library recompile against
// this header unchanged.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "audio_encoder.h"
#include "audio_injection.h"
#include "mel_spectrogram.h"
#include "qasr_capi.h"
#include "text_decoder.h"

namespace qwen3_asr {

// src/qwen3_asr.h:15-34
struct transcribe_params {
    int32_t max_tokens = 1024;
    std::string language = "";       // accepted, ignored (as src/qwen3_asr.cpp:211)
    std::string system_prompt = "";
    int32_t n_threads = 4;            // accepted for API compatibility (no host threads on the hot path)
    bool print_progress = false;
    bool print_timing = true;
};

// src/qwen3_asr.h:37-49
struct transcribe_result {
    std::string text;
    std::vector<int32_t> tokens;
    bool success = false;
    std::string error_msg;
    int64_t t_load_ms = 0;
    int64_t t_mel_ms = 0;
    int64_t t_encode_ms = 0;
    int64_t t_decode_ms = 0;   // prefill + greedy loop, as the reference's decode_greedy
    int64_t t_total_ms = 0;
};

using progress_callback_t = std::function<void(int tokens_generated, int max_tokens)>;

// src/qwen3_asr.h:55-116
class Qwen3ASR {
public:
    Qwen3ASR();
    ~Qwen3ASR();
    Qwen3ASR(const Qwen3ASR &) = delete;
    Qwen3ASR &operator=(const Qwen3ASR &) = delete;

    bool load_model(const std::string &model_path);
    transcribe_result transcribe(const std::string &audio_path, const transcribe_params &params = transcribe_params());
    transcribe_result transcribe(const float *samples, int n_samples, const transcribe_params &params = transcribe_params());
    void set_progress_callback(progress_callback_t callback);
    const std::string &get_error() const { return error_msg_; }
    bool is_loaded() const { return model_ != nullptr; }
    const text_decoder_config &get_config() const { return config_; }

    // MI355X additions: device selection, batched transcription, and the
    // --profile report (src/timing.h sections, device time, of the last call)
    void set_device(int device) { device_ = device; }
    // several clips: continuous batching over max_batch() KV-cache slots (a
    // finished clip's slot is refilled at once); results in input order, each
    // clip's success / error_msg its own
    std::vector<transcribe_result> transcribe_batch(const std::vector<std::vector<float>> &clips,
                                                    const transcribe_params &params = transcribe_params());
    // a work queue: fetch(id, pcm) -> false when empty (called whenever a slot
    // frees; a counter shared by several Qwen3ASR objects, one per device,
    // balances them dynamically); sink(id, result) as each clip finishes.
    // n_ctx: the context length (0: a 30 s clip's prompt + max_tokens);
    // slots: 0 = max_batch().  false: the run itself failed (get_error()).
    // Per clip only t_total_ms is set (its completion time within the stream:
    // the stages of different clips overlap); the progress callback sees
    // every clip's running count; --profile's report covers the whole stream.
    bool transcribe_stream(const std::function<bool(int &id, std::vector<float> &pcm)> &fetch,
                           const std::function<void(int id, transcribe_result result)> &sink,
                           const transcribe_params &params = transcribe_params(), int n_ctx = 0, int slots = 0);
    void set_max_batch(int slots) { max_batch_ = slots > 0 ? slots : 1; }
    int max_batch() const { return max_batch_; }
    void set_profile(bool on) { profile_ = on; }
    const std::string &profile_report() const { return profile_report_; }

private:
    transcribe_result transcribe_internal(const float *samples, int n_samples, const transcribe_params &params);
    bool ensure_ctx(int batch, int n_ctx);
    std::vector<transcribe_result> transcribe_run(const std::vector<std::vector<float>> &clips, const transcribe_params &params);

    qasr_model *model_ = nullptr;
    qasr_ctx *ctx_ = nullptr;
    int ctx_batch_ = 0, ctx_len_ = 0, device_ = 0, max_batch_ = 16;
    text_decoder_config config_;
    std::string error_msg_;
    progress_callback_t progress_callback_;
    bool profile_ = false;
    std::string profile_report_;
};

bool load_audio_file(const std::string &path, std::vector<float> &samples, int &sample_rate);

}  // namespace qwen3_asr
