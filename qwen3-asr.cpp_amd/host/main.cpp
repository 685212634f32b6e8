// main.cpp -- qwen3-asr-cli: the three modes of src/main.cpp (transcription
// :361-414, forced alignment --align :301-359, transcribe + align -a :416-500)
// with the same flags and output, plus MI355X additions: --device, batch file
// lists (-f may repeat, --file-list, transcription mode), --devices to shard a
// file list over several GPUs (one host thread and model replica per GPU,
// longest-first assignment: the sharded counterpart of the reference's shell
// loop, docs/usage.md:240-252), --synthetic to write a synthetic GGUF
// (tiny|full|aligner|aligner-tiny) for testing.
#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <sys/stat.h>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "forced_aligner.h"
#include "qasr_capi.h"
#include "qwen3_asr.h"

struct cli_params {
    std::string model_path = "models/qwen3-asr-0.6b-f16.gguf";
    std::string aligner_model_path;
    std::vector<std::string> audio_paths;
    std::string output_path, language, synthetic, align_text;
    int32_t max_tokens = 1024, n_threads = 4, device = 0, batch = 16;
    std::vector<int> devices;   // --devices: shard the files over these GPUs
    bool print_progress = false, print_timing = true, print_tokens = false, profile = false;
    bool align_mode = false, transcribe_align_mode = false;
};

static void usage(const char *prog) {
    fprintf(stderr, "Usage: %s [options]\n\nOptions:\n", prog);
    fprintf(stderr, "  -m, --model <path>     Path to GGUF model (default: models/qwen3-asr-0.6b-f16.gguf)\n");
    fprintf(stderr, "  -f, --audio <path>     Path to audio file (WAV, 16kHz mono) [required; repeat for a batch]\n");
    fprintf(stderr, "  -o, --output <path>    Output file path (default: stdout)\n");
    fprintf(stderr, "  -l, --language <code>  Language code (optional, e.g. 'korean' for Korean word splitting)\n");
    fprintf(stderr, "  -t, --threads <n>      Number of threads (accepted for compatibility)\n");
    fprintf(stderr, "  --max-tokens <n>       Maximum tokens to generate (default: 1024)\n");
    fprintf(stderr, "  --progress             Print progress during transcription\n");
    fprintf(stderr, "  --no-timing            Don't print timing information\n");
    fprintf(stderr, "  --tokens               Print token IDs\n");
    fprintf(stderr, "  --profile              Print timing profile\n");
    fprintf(stderr, "  --device <n>           HIP device index (default: 0)\n");
    fprintf(stderr, "  --file-list <path>     Text file with one audio path per line (added to the -f files)\n");
    fprintf(stderr, "  --devices <i,j,...>    Shard the audio files over these HIP devices (one replica each)\n");
    fprintf(stderr, "  --batch <n>            KV-cache slots per GPU (continuous batching) with --devices / several files (default: 16)\n");
    fprintf(stderr, "  --synthetic <cfg>      Write a synthetic GGUF (tiny|full|aligner|aligner-tiny) to --model and exit\n");
    fprintf(stderr, "\nForced Alignment:\n");
    fprintf(stderr, "  --align                Enable forced alignment mode\n");
    fprintf(stderr, "  --text <text>          Reference transcript for alignment\n");
    fprintf(stderr, "\nTranscribe + Align:\n");
    fprintf(stderr, "  -a, --transcribe-align Run ASR then forced alignment\n");
    fprintf(stderr, "  --aligner-model <path> Path to forced aligner GGUF model (required with --transcribe-align)\n");
    fprintf(stderr, "\n  -h, --help             Show this help message\n");
}

static bool parse(int argc, char **argv, cli_params &p) {
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        auto val = [&](std::string &dst) {
            if (i + 1 >= argc) { fprintf(stderr, "Error: %s requires an argument\n", a); return false; }
            dst = argv[++i];
            return true;
        };
        std::string v;
        if (!strcmp(a, "-m") || !strcmp(a, "--model")) { if (!val(p.model_path)) return false; }
        else if (!strcmp(a, "-f") || !strcmp(a, "--audio")) { if (!val(v)) return false; p.audio_paths.push_back(v); }
        else if (!strcmp(a, "-o") || !strcmp(a, "--output")) { if (!val(p.output_path)) return false; }
        else if (!strcmp(a, "-l") || !strcmp(a, "--language") || !strcmp(a, "--lang")) { if (!val(p.language)) return false; }
        else if (!strcmp(a, "-t") || !strcmp(a, "--threads")) { if (!val(v)) return false; p.n_threads = atoi(v.c_str()); }
        else if (!strcmp(a, "--max-tokens")) { if (!val(v)) return false; p.max_tokens = atoi(v.c_str()); }
        else if (!strcmp(a, "--device")) { if (!val(v)) return false; p.device = atoi(v.c_str()); }
        else if (!strcmp(a, "--batch")) { if (!val(v)) return false; p.batch = std::max(1, atoi(v.c_str())); }
        else if (!strcmp(a, "--devices")) {
            if (!val(v)) return false;
            for (size_t k = 0; k < v.size();) {
                const size_t e = v.find(',', k);
                p.devices.push_back(atoi(v.substr(k, e == std::string::npos ? std::string::npos : e - k).c_str()));
                if (e == std::string::npos) break;
                k = e + 1;
            }
        }
        else if (!strcmp(a, "--file-list")) {
            if (!val(v)) return false;
            std::ifstream f(v);
            if (!f) { fprintf(stderr, "Error: cannot read file list %s\n", v.c_str()); return false; }
            for (std::string line; std::getline(f, line);) {
                while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
                if (!line.empty()) p.audio_paths.push_back(line);
            }
        }
        else if (!strcmp(a, "--synthetic")) { if (!val(p.synthetic)) return false; }
        else if (!strcmp(a, "--progress")) p.print_progress = true;
        else if (!strcmp(a, "--no-timing")) p.print_timing = false;
        else if (!strcmp(a, "--tokens")) p.print_tokens = true;
        else if (!strcmp(a, "--profile")) p.profile = true;
        else if (!strcmp(a, "--align")) p.align_mode = true;
        else if (!strcmp(a, "-a") || !strcmp(a, "--transcribe-align")) p.transcribe_align_mode = true;
        else if (!strcmp(a, "--aligner-model")) { if (!val(p.aligner_model_path)) return false; }
        else if (!strcmp(a, "--text")) { if (!val(p.align_text)) return false; }
        else if (!strcmp(a, "-h") || !strcmp(a, "--help")) { usage(argv[0]); exit(0); }
        else { fprintf(stderr, "Error: Unknown argument: %s\n", a); return false; }
    }
    if (!p.synthetic.empty()) return true;
    if (p.audio_paths.empty()) { fprintf(stderr, "Error: Audio file path is required (-f/--audio)\n"); return false; }
    // src/main.cpp:76-90
    if (p.align_mode && p.align_text.empty()) {
        fprintf(stderr, "Error: Reference text is required for alignment mode (--text)\n");
        return false;
    }
    if (p.align_mode && p.transcribe_align_mode) {
        fprintf(stderr, "Error: --align and --transcribe-align cannot be used together\n");
        return false;
    }
    if (p.transcribe_align_mode && p.aligner_model_path.empty()) {
        fprintf(stderr, "Error: --aligner-model is required for --transcribe-align\n");
        return false;
    }
    if ((p.align_mode || p.transcribe_align_mode) && p.audio_paths.size() != 1) {
        fprintf(stderr, "Error: alignment takes exactly one audio file\n");
        return false;
    }
    return true;
}

// src/main.cpp:163-189: "language Xxxx..." prefix of the ASR text
static std::string detect_language(const std::string &asr_text) {
    const std::string prefix = "language ";
    if (asr_text.size() < prefix.size() || asr_text.compare(0, prefix.size(), prefix) != 0) return "";
    size_t pos = prefix.size();
    if (pos >= asr_text.size() || !std::isupper((unsigned char)asr_text[pos])) return "";
    ++pos;
    while (pos < asr_text.size() && std::islower((unsigned char)asr_text[pos])) ++pos;
    std::string lang = asr_text.substr(prefix.size(), pos - prefix.size());
    std::transform(lang.begin(), lang.end(), lang.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return lang;
}

// src/main.cpp:191-228
static std::string extract_transcript(const std::string &asr_text) {
    const std::string prefix = "language ";
    if (asr_text.size() < prefix.size() || asr_text.compare(0, prefix.size(), prefix) != 0) return asr_text;
    size_t pos = prefix.size();
    if (pos >= asr_text.size()) return "";
    if (!std::isupper((unsigned char)asr_text[pos])) return asr_text;
    ++pos;
    while (pos < asr_text.size() && std::islower((unsigned char)asr_text[pos])) ++pos;
    while (pos < asr_text.size()) {
        const unsigned char c = (unsigned char)asr_text[pos];
        if (c >= 0x80 || !std::isspace(c)) break;
        ++pos;
    }
    return asr_text.substr(pos);
}

// src/main.cpp:230-276
static std::string escape_json_string(const std::string &s) {
    std::string r;
    for (char c : s) {
        switch (c) {
            case '"': r += "\\\""; break;
            case '\\': r += "\\\\"; break;
            case '\b': r += "\\b"; break;
            case '\f': r += "\\f"; break;
            case '\n': r += "\\n"; break;
            case '\r': r += "\\r"; break;
            case '\t': r += "\\t"; break;
            default:
                if ((unsigned char)c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", (unsigned char)c); r += b; }
                else r += c;
        }
    }
    return r;
}

static std::string alignment_to_json(const qwen3_asr::alignment_result &result) {
    std::string json = "{\n  \"words\": [\n";
    for (size_t i = 0; i < result.words.size(); ++i) {
        const auto &w = result.words[i];
        char buf[64];
        snprintf(buf, sizeof buf, "\"start\": %.3f, \"end\": %.3f}", w.start, w.end);
        json += "    {\"word\": \"" + escape_json_string(w.word) + "\", " + buf;
        if (i + 1 < result.words.size()) json += ",";
        json += "\n";
    }
    json += "  ]\n}";
    return json;
}

// src/main.cpp:278-299
static std::string find_korean_dict(const std::string &model_path) {
    auto dir_of = [](const std::string &path) -> std::string {
        const size_t pos = path.find_last_of("/\\");
        return pos != std::string::npos ? path.substr(0, pos) : ".";
    };
    for (const std::string &p : {dir_of(model_path) + "/../assets/korean_dict_jieba.dict",
                                 dir_of(model_path) + "/assets/korean_dict_jieba.dict", std::string("assets/korean_dict_jieba.dict")}) {
        std::ifstream f(p);
        if (f.good()) return p;
    }
    return "";
}

static int write_output(const cli_params &p, const std::string &text) {
    if (p.output_path.empty()) {
        printf("%s", text.c_str());
        return 0;
    }
    std::ofstream out(p.output_path);
    if (!out) { fprintf(stderr, "Error: Failed to open output file: %s\n", p.output_path.c_str()); return 1; }
    out << text;
    fprintf(stderr, "Output written to: %s\n", p.output_path.c_str());
    return 0;
}

static bool load_aligner(qwen3_asr::ForcedAligner &al, const std::string &path, const std::string &lang, int device) {
    al.set_device(device);
    if (!al.load_model(path)) { fprintf(stderr, "Error (Aligner): %s\n", al.get_error().c_str()); return false; }
    if (lang == "korean") {
        const std::string dict = find_korean_dict(path);
        if (dict.empty()) fprintf(stderr, "Warning: Korean dictionary not found. Falling back to whitespace splitting.\n");
        else if (!al.load_korean_dict(dict)) fprintf(stderr, "Warning: Failed to load Korean dictionary from %s\n", dict.c_str());
    }
    return true;
}

static int run_alignment(const cli_params &p) {
    fprintf(stderr, "qwen3-asr-cli (Forced Alignment Mode)\n  Model: %s\n  Audio: %s\n  Text: %s\n", p.model_path.c_str(),
            p.audio_paths[0].c_str(), p.align_text.c_str());
    if (!p.language.empty()) fprintf(stderr, "  Language: %s\n", p.language.c_str());
    fprintf(stderr, "\n");
    qwen3_asr::ForcedAligner al;
    if (!load_aligner(al, p.model_path, p.language, p.device)) return 1;
    fprintf(stderr, "Model loaded. Running alignment...\n");
    auto r = al.align(p.audio_paths[0], p.align_text, p.language);
    if (!r.success) { fprintf(stderr, "Error: %s\n", r.error_msg.c_str()); return 1; }
    if (p.print_timing) {
        fprintf(stderr, "\nTiming:\n");
        fprintf(stderr, "  Mel spectrogram: %lld ms\n", (long long)r.t_mel_ms);
        fprintf(stderr, "  Audio encoding:  %lld ms\n", (long long)r.t_encode_ms);
        fprintf(stderr, "  Text decoding:   %lld ms\n", (long long)r.t_decode_ms);
        fprintf(stderr, "  Total:           %lld ms\n", (long long)r.t_total_ms);
        fprintf(stderr, "  Words aligned:   %zu\n", r.words.size());
    }
    return write_output(p, alignment_to_json(r) + "\n");
}

static int run_transcribe_and_align(const cli_params &p) {
    fprintf(stderr, "qwen3-asr-cli (Transcribe + Align Mode)\n  ASR Model: %s\n  Aligner Model: %s\n  Audio: %s\n  Threads: %d\n\n",
            p.model_path.c_str(), p.aligner_model_path.c_str(), p.audio_paths[0].c_str(), p.n_threads);
    fprintf(stderr, "--- Phase 1: Transcription ---\n");
    qwen3_asr::Qwen3ASR asr;
    asr.set_device(p.device);
    if (!asr.load_model(p.model_path)) { fprintf(stderr, "Error (ASR): %s\n", asr.get_error().c_str()); return 1; }
    qwen3_asr::transcribe_params tp;
    tp.max_tokens = p.max_tokens;
    tp.language = p.language;
    tp.n_threads = p.n_threads;
    tp.print_progress = p.print_progress;
    tp.print_timing = p.print_timing;
    auto ar = asr.transcribe(p.audio_paths[0], tp);
    if (!ar.success) { fprintf(stderr, "Error (ASR): %s\n", ar.error_msg.c_str()); return 1; }
    const std::string detected = detect_language(ar.text);
    const std::string lang = p.language.empty() ? detected : p.language;
    const std::string transcript = extract_transcript(ar.text);
    fprintf(stderr, "  Detected language: %s\n", detected.empty() ? "(none)" : detected.c_str());
    if (!p.language.empty()) fprintf(stderr, "  Language override: %s\n", p.language.c_str());
    fprintf(stderr, "  Alignment language: %s\n", lang.empty() ? "(none)" : lang.c_str());
    fprintf(stderr, "  Transcript: %s\n", transcript.c_str());
    fprintf(stderr, "\n--- Phase 2: Forced Alignment ---\n");
    qwen3_asr::ForcedAligner al;
    if (!load_aligner(al, p.aligner_model_path, lang, p.device)) return 1;
    auto r = al.align(p.audio_paths[0], transcript, lang);
    if (!r.success) { fprintf(stderr, "Error (Aligner): %s\n", r.error_msg.c_str()); return 1; }
    if (p.print_timing) {
        fprintf(stderr, "\nCombined Timing:\n");
        fprintf(stderr, "  ASR:           %lld ms\n", (long long)ar.t_total_ms);
        fprintf(stderr, "  Alignment:     %lld ms\n", (long long)r.t_total_ms);
        fprintf(stderr, "  Total:         %lld ms\n", (long long)(ar.t_total_ms + r.t_total_ms));
        fprintf(stderr, "  Words aligned: %zu\n", r.words.size());
    }
    return write_output(p, alignment_to_json(r) + "\n");
}

// --devices: one host thread per GPU, each with its own model replica and
// context (the reference's objects are single-threaded; so are ours), pulling
// files from one shared queue (longest first) into its continuous-batching
// stream of --batch slots: a device that finishes early takes the next file,
// so the tail stays balanced whatever the decode lengths; output in input order
static int run_transcription_sharded(const cli_params &p) {
    const size_t N = p.audio_paths.size();
    const int G = (int)p.devices.size();
    std::vector<long long> size(N);
    for (size_t i = 0; i < N; i++) {
        struct stat st;
        size[i] = stat(p.audio_paths[i].c_str(), &st) == 0 ? (long long)st.st_size : 0;
    }
    std::vector<size_t> order(N);
    for (size_t i = 0; i < N; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return size[a] > size[b]; });
    fprintf(stderr, "qwen3-asr-cli (sharded)\n  Model: %s\n  Files: %zu over %d GPU(s), %d slots each, shared queue\n\n",
            p.model_path.c_str(), N, G, p.batch);
    // the stream's context: the longest file's prompt + the budget (16-bit PCM:
    // at most size / 2 samples), capped at kStreamSecs of audio -- every slot
    // gets that length, so one long file must not multiply the whole cache
    // (ADVICE r4).  Longer files go to a second queue that the device threads
    // take one at a time after their streams, each in a context sized to that
    // file as the reference sizes its context per clip (src/qwen3_asr.cpp:223).
    constexpr long long kStreamSecs = 120;
    std::vector<size_t> longq;
    while (!order.empty() && size[order.front()] / 2 > kStreamSecs * 16000) {
        longq.push_back(order.front());
        order.erase(order.begin());
    }
    const size_t NS = order.size();
    const long long max_samples = NS ? size[order[0]] / 2 : 0;
    const int n_ctx = qasr_prompt_len(qasr_encoder_frames(qasr_mel_frames((int)std::min<long long>(max_samples, 1LL << 30)))) +
                      p.max_tokens + 64;
    std::atomic<size_t> next_long{0};
    std::vector<qwen3_asr::transcribe_result> results(N);
    std::vector<std::string> errors(G);
    std::atomic<size_t> next{0};
    std::atomic<long long> samples{0};
    std::mutex res_mu;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++) {
        th.emplace_back([&, g] {
            qwen3_asr::Qwen3ASR asr;
            asr.set_device(p.devices[g]);
            asr.set_max_batch(p.batch);
            if (!asr.load_model(p.model_path)) { errors[g] = asr.get_error(); return; }
            qwen3_asr::transcribe_params tp;
            tp.max_tokens = p.max_tokens;
            tp.language = p.language;
            tp.print_timing = false;
            auto fetch = [&](int &id, std::vector<float> &pcm) {
                for (;;) {
                    const size_t k = next++;
                    if (k >= NS) return false;
                    const size_t i = order[k];
                    int sr = 0;
                    if (qwen3_asr::load_audio_file(p.audio_paths[i], pcm, sr) && sr == 16000) {
                        samples += (long long)pcm.size();
                        id = (int)i;
                        return true;
                    }
                    std::lock_guard<std::mutex> lk(res_mu);   // this file fails alone
                    results[i].error_msg = "Failed to load audio file: " + p.audio_paths[i];
                }
            };
            auto sink = [&](int id, qwen3_asr::transcribe_result r) {
                std::lock_guard<std::mutex> lk(res_mu);
                results[id] = std::move(r);
            };
            if (NS && !asr.transcribe_stream(fetch, sink, tp, n_ctx)) { errors[g] = asr.get_error(); return; }
            for (size_t k; (k = next_long++) < longq.size();) {   // files past the stream's cap, one at a time
                const size_t i = longq[k];
                qwen3_asr::transcribe_result r = asr.transcribe(p.audio_paths[i], tp);
                std::lock_guard<std::mutex> lk(res_mu);
                if (r.success) samples += size[i] / 2;
                results[i] = std::move(r);
            }
        });
    }
    for (auto &t : th) t.join();
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int g = 0; g < G; g++)
        if (!errors[g].empty()) { fprintf(stderr, "Error (device %d): %s\n", p.devices[g], errors[g].c_str()); return 1; }
    std::string all;
    for (size_t i = 0; i < N; i++) {
        if (!results[i].success) { fprintf(stderr, "Error (%s): %s\n", p.audio_paths[i].c_str(), results[i].error_msg.c_str()); return 1; }
        all += results[i].text + "\n";
    }
    if (p.print_timing)
        fprintf(stderr, "Sharded timing: %.1f s of audio in %.3f s over %d GPU(s) (RTFx %.1f, model loads included)\n",
                samples.load() / 16000.0, wall, G, samples.load() / 16000.0 / wall);
    return write_output(p, all);
}

static int run_transcription(const cli_params &p) {
    fprintf(stderr, "qwen3-asr-cli\n  Model: %s\n", p.model_path.c_str());
    for (auto &a : p.audio_paths) fprintf(stderr, "  Audio: %s\n", a.c_str());
    fprintf(stderr, "  Threads: %d\n\n", p.n_threads);
    qwen3_asr::Qwen3ASR asr;
    asr.set_device(p.device);
    asr.set_profile(p.profile);
    if (!asr.load_model(p.model_path)) { fprintf(stderr, "Error: %s\n", asr.get_error().c_str()); return 1; }
    qwen3_asr::transcribe_params tp;
    tp.max_tokens = p.max_tokens;
    tp.language = p.language;
    tp.n_threads = p.n_threads;
    tp.print_progress = p.print_progress;
    tp.print_timing = p.print_timing;
    std::vector<qwen3_asr::transcribe_result> results;
    if (p.audio_paths.size() == 1) {
        results.push_back(asr.transcribe(p.audio_paths[0], tp));
    } else {
        std::vector<std::vector<float>> clips;
        for (auto &a : p.audio_paths) {
            std::vector<float> s;
            int sr = 0;
            if (!qwen3_asr::load_audio_file(a, s, sr) || sr != 16000) { fprintf(stderr, "Error: bad audio %s\n", a.c_str()); return 1; }
            clips.push_back(std::move(s));
        }
        asr.set_max_batch(p.batch);
        results = asr.transcribe_batch(clips, tp);
    }
    std::string all;
    for (const auto &r : results) {
        if (!r.success) { fprintf(stderr, "Error: %s\n", r.error_msg.c_str()); return 1; }
        if (p.print_tokens) {
            fprintf(stderr, "\nTokens (%zu):\n", r.tokens.size());
            for (size_t k = 0; k < r.tokens.size(); ++k) fprintf(stderr, "  [%zu] %d\n", k, r.tokens[k]);
            fprintf(stderr, "\n");
        }
        all += r.text + "\n";
    }
    const int rc = write_output(p, all);
    if (p.profile) fprintf(stderr, "%s", asr.profile_report().c_str());   // src/main.cpp:409-411
    return rc;
}

int main(int argc, char **argv) {
    cli_params p;
    if (!parse(argc, argv, p)) { fprintf(stderr, "\n"); usage(argv[0]); return 1; }
    if (!p.synthetic.empty()) {
        if (qasr_write_synthetic_gguf(p.model_path.c_str(), p.synthetic.c_str(), 42, 1) != 0) {
            fprintf(stderr, "Error: %s\n", qasr_last_error());
            return 1;
        }
        fprintf(stderr, "wrote synthetic %s model to %s\n", p.synthetic.c_str(), p.model_path.c_str());
        return 0;
    }
    if (p.transcribe_align_mode) return run_transcribe_and_align(p);
    if (p.align_mode) return run_alignment(p);
    if (!p.devices.empty()) return run_transcription_sharded(p);
    return run_transcription(p);
}
