// timing.h -- the reference's QWEN3_TIMER section-timer macros
// (src/timing.h:12-72) for callers that instrument their own code around the
// API: with QWEN3_ASR_TIMING defined, QWEN3_TIMER(name) times the enclosing
// scope on the host clock into a process-wide table, QWEN3_TIMER_RESET()
// clears it and QWEN3_TIMER_REPORT() prints it to stderr in the reference's
// layout; without it the macros compile to nothing.  The engine's own
// sections (mel_spectrogram, audio_encoding.*, decode.*) are timed on the
// device with HIP events and reported by qasr_profile_report /
// Qwen3ASR::profile_report (the CLI's --profile) in the same layout.
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>

namespace qwen3_asr {

#ifdef QWEN3_ASR_TIMING

class TimingProfiler {
public:
    static TimingProfiler &instance() {
        static TimingProfiler p;
        return p;
    }
    void record(const std::string &name, int64_t us) {
        std::lock_guard<std::mutex> lk(mu_);
        auto &e = table_[name];
        e.first += us;
        e.second += 1;
    }
    void reset() {
        std::lock_guard<std::mutex> lk(mu_);
        table_.clear();
    }
    void print_report() const {
        std::lock_guard<std::mutex> lk(mu_);
        const char *rule = "================================================================================";
        std::fprintf(stderr, "\n%s\n%*s\n%s\n", rule, 53, "TIMING PROFILE REPORT", rule);
        std::fprintf(stderr, "%-45s %12s %8s %12s\n", "Section", "Total (ms)", "Calls", "Avg (ms)");
        std::fprintf(stderr, "--------------------------------------------------------------------------------\n");
        for (const auto &kv : table_) {
            const double ms = kv.second.first / 1000.0;
            const long long n = kv.second.second;
            std::fprintf(stderr, "%-45s %12.2f %8lld %12.2f\n", kv.first.c_str(), ms, n, n ? ms / n : 0.0);
        }
        std::fprintf(stderr, "%s\n", rule);
    }

private:
    TimingProfiler() = default;
    mutable std::mutex mu_;
    std::map<std::string, std::pair<int64_t, int64_t>> table_;   // total us, calls
};

class ScopedTimer {
public:
    explicit ScopedTimer(std::string name) : name_(std::move(name)), t0_(std::chrono::steady_clock::now()) {}
    ~ScopedTimer() {
        const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0_).count();
        TimingProfiler::instance().record(name_, us);
    }
    ScopedTimer(const ScopedTimer &) = delete;
    ScopedTimer &operator=(const ScopedTimer &) = delete;

private:
    std::string name_;
    std::chrono::steady_clock::time_point t0_;
};

#define QWEN3_TIMER_CAT2(a, b) a##b
#define QWEN3_TIMER_CAT(a, b) QWEN3_TIMER_CAT2(a, b)
#define QWEN3_TIMER(name) qwen3_asr::ScopedTimer QWEN3_TIMER_CAT(qwen3_timer_, __LINE__)(name)
#define QWEN3_TIMER_RESET() qwen3_asr::TimingProfiler::instance().reset()
#define QWEN3_TIMER_REPORT() qwen3_asr::TimingProfiler::instance().print_report()

#else

#define QWEN3_TIMER(name) ((void)0)
#define QWEN3_TIMER_RESET() ((void)0)
#define QWEN3_TIMER_REPORT() ((void)0)

#endif

}  // namespace qwen3_asr
