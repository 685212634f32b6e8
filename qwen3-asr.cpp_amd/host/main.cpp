// main.cpp -- qwen3-asr-cli, transcription mode of src/main.cpp:14-161, 361-414
// (same flags and output), plus MI355X additions: --device, batch file lists
// (-f may repeat), --synthetic to write a synthetic GGUF for testing.
// Forced alignment (--align / --transcribe-align) is the SURVEY §8(f) "next"
// row and is rejected with a clear message in this build.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "qwen3_asr.h"

struct cli_params {
    std::string model_path = "models/qwen3-asr-0.6b-f16.gguf";
    std::vector<std::string> audio_paths;
    std::string output_path, language, synthetic;
    int32_t max_tokens = 1024, n_threads = 4, device = 0;
    bool print_progress = false, print_timing = true, print_tokens = false, profile = false, align = false;
};

static void usage(const char *prog) {
    fprintf(stderr, "Usage: %s [options]\n\nOptions:\n", prog);
    fprintf(stderr, "  -m, --model <path>     Path to GGUF model (default: models/qwen3-asr-0.6b-f16.gguf)\n");
    fprintf(stderr, "  -f, --audio <path>     Path to audio file (WAV, 16kHz mono) [required; repeat for a batch]\n");
    fprintf(stderr, "  -o, --output <path>    Output file path (default: stdout)\n");
    fprintf(stderr, "  -l, --language <code>  Language code (accepted, ignored by the ASR path)\n");
    fprintf(stderr, "  -t, --threads <n>      Number of threads (accepted for compatibility)\n");
    fprintf(stderr, "  --max-tokens <n>       Maximum tokens to generate (default: 1024)\n");
    fprintf(stderr, "  --progress             Print progress during transcription\n");
    fprintf(stderr, "  --no-timing            Don't print timing information\n");
    fprintf(stderr, "  --tokens               Print token IDs\n");
    fprintf(stderr, "  --profile              Print timing profile\n");
    fprintf(stderr, "  --device <n>           HIP device index (default: 0)\n");
    fprintf(stderr, "  --synthetic <cfg>      Write a synthetic GGUF (tiny|full) to --model and exit\n");
    fprintf(stderr, "  -h, --help             Show this help message\n");
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
        else if (!strcmp(a, "--synthetic")) { if (!val(p.synthetic)) return false; }
        else if (!strcmp(a, "--progress")) p.print_progress = true;
        else if (!strcmp(a, "--no-timing")) p.print_timing = false;
        else if (!strcmp(a, "--tokens")) p.print_tokens = true;
        else if (!strcmp(a, "--profile")) p.profile = true;
        else if (!strcmp(a, "--align") || !strcmp(a, "-a") || !strcmp(a, "--transcribe-align") || !strcmp(a, "--aligner-model") ||
                 !strcmp(a, "--text")) {
            p.align = true;
            if (strcmp(a, "--align") && strcmp(a, "-a") && strcmp(a, "--transcribe-align") && i + 1 < argc) ++i;
        } else if (!strcmp(a, "-h") || !strcmp(a, "--help")) { usage(argv[0]); exit(0); }
        else { fprintf(stderr, "Error: Unknown argument: %s\n", a); return false; }
    }
    if (p.align) { fprintf(stderr, "Error: forced alignment is not available in this build (ASR path only)\n"); return false; }
    if (p.synthetic.empty() && p.audio_paths.empty()) { fprintf(stderr, "Error: Audio file path is required (-f/--audio)\n"); return false; }
    return true;
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
    fprintf(stderr, "qwen3-asr-cli\n  Model: %s\n", p.model_path.c_str());
    for (auto &a : p.audio_paths) fprintf(stderr, "  Audio: %s\n", a.c_str());
    fprintf(stderr, "  Threads: %d\n\n", p.n_threads);
    qwen3_asr::Qwen3ASR asr;
    asr.set_device(p.device);
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
        results = asr.transcribe_batch(clips, tp);
    }
    std::string all;
    for (size_t i = 0; i < results.size(); i++) {
        const auto &r = results[i];
        if (!r.success) { fprintf(stderr, "Error: %s\n", r.error_msg.c_str()); return 1; }
        if (p.print_tokens) {
            fprintf(stderr, "\nTokens (%zu):\n", r.tokens.size());
            for (size_t k = 0; k < r.tokens.size(); ++k) fprintf(stderr, "  [%zu] %d\n", k, r.tokens[k]);
            fprintf(stderr, "\n");
        }
        all += r.text + "\n";
    }
    if (p.output_path.empty()) {
        printf("%s", all.c_str());
    } else {
        std::ofstream out(p.output_path);
        if (!out) { fprintf(stderr, "Error: Failed to open output file: %s\n", p.output_path.c_str()); return 1; }
        out << all;
        fprintf(stderr, "Output written to: %s\n", p.output_path.c_str());
    }
    return 0;
}
