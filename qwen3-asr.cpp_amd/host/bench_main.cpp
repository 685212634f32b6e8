// bench_main.cpp -- qasr-bench: the bench.py workload as a native program.
//
// Same work as bench.py at N = 1 (synthetic full-size GGUF, seeded clips
// qasr_synth_pcm(1000 + i), PCM staged in HBM, W warmup + K timed qasr_run
// calls with a fixed decode budget, EOS ignored).  It exists for profilers
// that cannot attach to the Python process (rocprofv3 --pmc faults inside a
// ctypes-driven HIP launch on this image; the CLI and this binary are fine),
// so the PMC passes under profiles/ measure exactly the bench kernels.
//
//   qasr-bench [--model M.gguf] [--seconds 92] [--batch 1] [--steps K]
//              [--warmup W] [--tok-rate 3.5] [--q8]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "qasr_capi.h"

static int die(const char *what) {
    fprintf(stderr, "qasr-bench: %s: %s\n", what, qasr_last_error());
    return 1;
}

int main(int argc, char **argv) {
    std::string model;
    double seconds = 92.0, tok_rate = 3.5;
    int batch = 1, steps = 2, warmup = 1, wtype = 1;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : nullptr;
        if (!strcmp(a, "--model") && v) { model = v; i++; }
        else if (!strcmp(a, "--seconds") && v) { seconds = atof(v); i++; }
        else if (!strcmp(a, "--batch") && v) { batch = atoi(v); i++; }
        else if (!strcmp(a, "--steps") && v) { steps = atoi(v); i++; }
        else if (!strcmp(a, "--warmup") && v) { warmup = atoi(v); i++; }
        else if (!strcmp(a, "--tok-rate") && v) { tok_rate = atof(v); i++; }
        else if (!strcmp(a, "--q8")) wtype = 8;
        else { fprintf(stderr, "qasr-bench: unknown argument %s\n", a); return 2; }
    }
    if (batch < 1 || steps < 1 || warmup < 0 || seconds <= 0) { fprintf(stderr, "qasr-bench: bad arguments\n"); return 2; }
    if (model.empty()) {
        const char *td = getenv("TMPDIR");
        model = std::string(td ? td : "/tmp") + (wtype == 8 ? "/qasr_synth_full_q8_0.gguf" : "/qasr_synth_full_f16.gguf");
        struct stat st;
        if (stat(model.c_str(), &st) != 0 && qasr_write_synthetic_gguf(model.c_str(), "full", 42, wtype)) return die("write model");
    }
    qasr_model *m = nullptr;
    qasr_ctx *c = nullptr;
    if (qasr_model_load(model.c_str(), 0, &m)) return die("model load");
    const int n = (int)(seconds * 16000);
    const int ntok = (int)std::ceil(tok_rate * seconds);
    const int P = qasr_prompt_len(qasr_encoder_frames(qasr_mel_frames(n)));
    if (qasr_ctx_create(m, batch, P + ntok + 8, &c)) return die("context");
    std::vector<std::vector<float>> clips(batch, std::vector<float>(n));
    std::vector<const float *> ptr(batch);
    std::vector<int> nn(batch, n);
    for (int b = 0; b < batch; b++) {
        qasr_synth_pcm(1000 + b, n, clips[b].data());
        ptr[b] = clips[b].data();
    }
    if (qasr_stage_audio(c, ptr.data(), nn.data(), batch)) return die("stage");
    std::vector<int32_t> toks((size_t)batch * ntok);
    std::vector<int> nt(batch);
    qasr_timings t{};
    for (int i = 0; i < warmup; i++)
        if (qasr_run(c, ntok, 1, toks.data(), nt.data(), &t)) return die("warmup");
    double mel = 0, enc = 0, pre = 0, dec = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; i++) {
        if (qasr_run(c, ntok, 1, toks.data(), nt.data(), &t)) return die("run");
        mel += t.t_mel_ms; enc += t.t_encode_ms; pre += t.t_prefill_ms; dec += t.t_decode_ms;
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int b = 0; b < batch; b++)
        if (nt[b] != ntok) { fprintf(stderr, "qasr-bench: decode budget not met\n"); return 1; }
    printf("{\"rtfx\": %.3f, \"ms_per_step\": %.3f, \"decode_tokens_per_s\": %.2f, \"clips\": %d, \"seconds\": %g, "
           "\"tokens\": %d, \"stage_ms\": {\"mel\": %.3f, \"encode\": %.3f, \"prefill\": %.3f, \"decode\": %.3f}}\n",
           batch * seconds * steps / dt, dt / steps * 1e3, batch * (double)ntok * steps / dt, batch, seconds, ntok,
           mel / steps, enc / steps, pre / steps, dec / steps);
    qasr_ctx_free(c);
    qasr_model_free(m);
    return 0;
}
