// host_util.cpp -- host-side pieces: hparams, tables, WAV, BPE, prompt,
// synthetic GGUF.  Each function cites the reference behaviour it mirrors.
#include "qasr_host.h"

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

namespace qasr {

// ------------------------------------------------------------------ fp16
uint16_t f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);
    if (ax < 0x38800000u) {
        if (ax <= 0x33000000u) return (uint16_t)sign;
        uint32_t e = ax >> 23, mant = (ax & 0x7fffffu) | 0x800000u, sh = 126u - e;
        uint32_t q = mant >> sh, rem = mant & ((1u << sh) - 1u), half = 1u << (sh - 1);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t h = (ax - 0x38000000u) >> 13, rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

float f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) x = sign;
        else {
            int sh = 0;
            while (!(m & 0x400u)) { m <<= 1; sh++; }
            x = sign | ((uint32_t)(113 - sh) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) x = sign | 0x7f800000u | (m << 13);
    else x = sign | ((e + 112u) << 23) | (m << 13);
    float f;
    memcpy(&f, &x, 4);
    return f;
}

// --------------------------------------------------------------- hparams
static int64_t geti2(const GGUFFile &f, const char *k1, const char *k2, int64_t def) {
    if (f.find(k1)) return f.get_int(k1, def);
    if (k2 && f.find(k2)) return f.get_int(k2, def);
    return def;
}

Hparams read_hparams(const GGUFFile &f) {
    Hparams hp;
    hp.enc_layers = (int)geti2(f, "audio.encoder_layers", "qwen3-asr.audio.encoder.layer_count", 18);
    hp.d_model = (int)geti2(f, "audio.d_model", "qwen3-asr.audio.encoder.embedding_length", 896);
    hp.enc_heads = (int)geti2(f, "audio.attention_heads", "qwen3-asr.audio.encoder.attention.head_count", 14);
    hp.enc_ffn = (int)geti2(f, "audio.ffn_dim", "qwen3-asr.audio.encoder.feed_forward_length", 3584);
    hp.conv_ch = (int)geti2(f, "audio.conv_channels", "qwen3-asr.audio.conv_channels", 480);
    hp.n_mel = (int)geti2(f, "audio.num_mel_bins", "qwen3-asr.audio.num_mel_bins", 128);
    hp.enc_eps = (float)f.get_float("audio.layer_norm_eps", 1e-5);
    // text decoder: src/text_decoder.cpp:130-144 (eos/pad hard-coded :140-141)
    hp.vocab = (int)f.get_int("qwen3-asr.vocab_size", 151936);
    hp.hidden = (int)f.get_int("qwen3-asr.embedding_length", 1024);
    hp.dec_layers = (int)f.get_int("qwen3-asr.block_count", 28);
    hp.n_head = (int)f.get_int("qwen3-asr.attention.head_count", 16);
    hp.n_kv_head = (int)f.get_int("qwen3-asr.attention.head_count_kv", 8);
    hp.dec_ffn = (int)f.get_int("qwen3-asr.feed_forward_length", 3072);
    hp.head_dim = (int)f.get_int("qwen3-asr.attention.key_length", 128);
    hp.rms_eps = (float)f.get_float("qwen3-asr.attention.layer_norm_rms_epsilon", 1e-6);
    hp.rope_theta = (float)f.get_float("qwen3-asr.rope.freq_base", 1000000.0);
    hp.audio_start_id = (int)f.get_int("qwen3-asr.audio.start_token_id", 151669);
    hp.audio_end_id = (int)f.get_int("qwen3-asr.audio.end_token_id", 151670);
    hp.audio_pad_id = (int)f.get_int("qwen3-asr.audio.pad_token_id", 151676);
    const gguf_tensor *t = f.tensor("blk.0.attn_q.weight");
    hp.weight_type = t ? (int)t->type : 1;
    // ForcedAligner (src/forced_aligner.cpp:136-175): its loader reads the
    // converter's keys only, with its own defaults (24 x 1024 encoder, vocab 152064)
    const gguf_tensor *head = f.tensor("output.weight");
    if (f.find("qwen3-asr.classify_num") || head) {
        hp.aligner = true;
        hp.enc_layers = (int)f.get_int("qwen3-asr.audio.encoder.layer_count", 24);
        hp.d_model = (int)f.get_int("qwen3-asr.audio.encoder.embedding_length", 1024);
        hp.enc_heads = (int)f.get_int("qwen3-asr.audio.encoder.attention.head_count", 16);
        hp.enc_ffn = (int)f.get_int("qwen3-asr.audio.encoder.feed_forward_length", 4096);
        hp.n_mel = (int)f.get_int("qwen3-asr.audio.num_mel_bins", 128);
        hp.conv_ch = (int)f.get_int("qwen3-asr.audio.conv_channels", 480);
        hp.vocab = (int)f.get_int("qwen3-asr.vocab_size", 152064);
        hp.classify_num = (int)f.get_int("qwen3-asr.classify_num", 5000);
        hp.timestamp_id = (int)f.get_int("qwen3-asr.timestamp_token_id", 151705);
    }
    return hp;
}

// ---------------------------------------------------------------- tables
static float hz_to_mel(float hz) { return 2595.0f * log10f(1.0f + hz / 700.0f); }
static float mel_to_hz(float mel) { return 700.0f * (powf(10.0f, mel / 2595.0f) - 1.0f); }

void mel_filters(std::vector<float> &f, int n_mels, int n_fft, int sr) {
    const int nb = 1 + n_fft / 2;
    f.assign((size_t)n_mels * nb, 0.0f);
    const float mel_min = hz_to_mel(0.0f), mel_max = hz_to_mel(sr / 2.0f);
    std::vector<float> hz(n_mels + 2), bins(n_mels + 2);
    for (int i = 0; i < n_mels + 2; i++) {
        float mp = mel_min + (mel_max - mel_min) * i / (n_mels + 1);
        hz[i] = mel_to_hz(mp);
        bins[i] = (n_fft + 1) * hz[i] / sr;
    }
    for (int m = 0; m < n_mels; m++) {
        const float l = bins[m], c = bins[m + 1], r = bins[m + 2];
        for (int k = 0; k < nb; k++) {
            float w = 0.0f;
            if (k >= l && k <= c) w = (k - l) / (c - l);
            else if (k >= c && k <= r) w = (r - k) / (r - c);
            f[(size_t)m * nb + k] = w;
        }
        const float enorm = 2.0f / (hz[m + 2] - hz[m]);
        for (int k = 0; k < nb; k++) f[(size_t)m * nb + k] *= enorm;
    }
}

void sinusoidal_pe(std::vector<float> &pe, int n_ctx, int d) {
    const int half = d / 2;
    pe.assign((size_t)n_ctx * d, 0.0f);
    for (int pos = 0; pos < n_ctx; ++pos)
        for (int i = 0; i < half; ++i) {
            float div_term = expf(-logf(10000.0f) * i / (half - 1));
            float angle = pos * div_term;
            pe[(size_t)pos * d + i] = sinf(angle);
            pe[(size_t)pos * d + half + i] = cosf(angle);
        }
}

static float gelu_tanh(float x) {
    const float A = 0.044715f, S = 0.79788456080286535587989211986876f;
    return 0.5f * x * (1.0f + tanhf(S * x * (1.0f + A * x * x)));
}

void gelu_table(std::vector<uint16_t> &t) {
    t.resize(65536);
    for (int i = 0; i < 65536; i++) t[i] = f32_to_f16(gelu_tanh(f16_to_f32((uint16_t)i)));
}

void rope_table(std::vector<float> &cs, int n_pos, int hd, float base) {
    const int half = hd / 2;
    cs.assign((size_t)n_pos * half * 2, 0.0f);
    const float theta_scale = powf(base, -2.0f / hd);
    for (int p = 0; p < n_pos; p++) {
        float theta = (float)p;
        for (int i = 0; i < half; i++) {
            cs[((size_t)p * half + i) * 2 + 0] = cosf(theta);
            cs[((size_t)p * half + i) * 2 + 1] = sinf(theta);
            theta *= theta_scale;
        }
    }
}

void dft_twiddles(std::vector<double> &tw) {
    const int fs = 400, nb = 201;
    tw.resize((size_t)fs * nb * 2);
    for (int n = 0; n < fs; n++)
        for (int k = 0; k < nb; k++) {
            double angle = 2.0 * M_PI * k * n / fs;   // evaluated exactly as the reference loop
            tw[((size_t)n * nb + k) * 2 + 0] = cos(angle);
            tw[((size_t)n * nb + k) * 2 + 1] = sin(angle);
        }
}

void hann_window(std::vector<double> &w) {
    w.resize(400);
    for (int i = 0; i < 400; i++) w[i] = 0.5 * (1.0 - cos((2.0 * M_PI * i) / 400));
}

// ----------------------------------------------------------------- audio
int mel_frames(int n) { return n < 0 ? 0 : (n + 400 - 400) / 160 + 1 - 1; }
int chunk_out_len(int L) {
    for (int i = 0; i < 3; i++) L = (L - 1) / 2 + 1;
    return L;
}
int encoder_frames(int T) {
    int n = 0;
    for (int s = 0; s < T; s += 100) n += chunk_out_len(T - s < 100 ? T - s : 100);
    return n;
}

bool load_wav(const std::string &path, std::vector<float> &samples, int &sr_out, std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { err = "Cannot open WAV file: " + path; return false; }
    char id[4];
    uint32_t u32;
    f.read(id, 4);
    if (!f || memcmp(id, "RIFF", 4)) { err = "Not a valid WAV file (missing RIFF header)"; return false; }
    f.read((char *)&u32, 4);
    f.read(id, 4);
    if (!f || memcmp(id, "WAVE", 4)) { err = "Not a valid WAV file (missing WAVE header)"; return false; }
    uint16_t fmt = 0, nch = 0, bps = 0;
    uint32_t sr = 0;
    while (f.good()) {
        uint32_t sz = 0;
        f.read(id, 4);
        f.read((char *)&sz, 4);
        if (!f) break;
        if (!memcmp(id, "fmt ", 4)) {
            uint32_t br; uint16_t ba;
            f.read((char *)&fmt, 2); f.read((char *)&nch, 2); f.read((char *)&sr, 4);
            f.read((char *)&br, 4); f.read((char *)&ba, 2); f.read((char *)&bps, 2);
            if (sz > 16) f.seekg(sz - 16, std::ios::cur);
        } else if (!memcmp(id, "data", 4)) {
            if (fmt != 1) { err = "Only PCM format supported (got format " + std::to_string(fmt) + ")"; return false; }
            if (bps != 16) { err = "Only 16-bit samples supported (got " + std::to_string(bps) + " bits)"; return false; }
            if (nch == 0) { err = "WAV has zero channels"; return false; }
            sr_out = (int)sr;
            const size_t n = sz / 2 / nch;
            std::vector<int16_t> raw(n * nch);
            f.read((char *)raw.data(), (std::streamsize)(raw.size() * 2));
            samples.resize(n);
            for (size_t i = 0; i < n; i++) {
                if (nch == 1) samples[i] = raw[i] / 32768.0f;
                else {
                    float s = 0;
                    for (int c = 0; c < nch; c++) s += raw[i * nch + c];
                    samples[i] = (s / nch) / 32768.0f;
                }
            }
            return true;
        } else {
            f.seekg(sz, std::ios::cur);
        }
    }
    err = "No data chunk found in WAV file";
    return false;
}

bool write_wav(const std::string &path, const float *pcm, int n, int sr) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    uint32_t data = (uint32_t)n * 2, riff = 36 + data, fmt_sz = 16, br = (uint32_t)sr * 2;
    uint16_t pcm_fmt = 1, ch = 1, ba = 2, bps = 16;
    fwrite("RIFF", 1, 4, f); fwrite(&riff, 4, 1, f); fwrite("WAVE", 1, 4, f);
    fwrite("fmt ", 1, 4, f); fwrite(&fmt_sz, 4, 1, f); fwrite(&pcm_fmt, 2, 1, f); fwrite(&ch, 2, 1, f);
    fwrite(&sr, 4, 1, f); fwrite(&br, 4, 1, f); fwrite(&ba, 2, 1, f); fwrite(&bps, 2, 1, f);
    fwrite("data", 1, 4, f); fwrite(&data, 4, 1, f);
    for (int i = 0; i < n; i++) {
        float v = pcm[i] * 32768.0f;
        v = v > 32767.0f ? 32767.0f : (v < -32768.0f ? -32768.0f : v);
        int16_t s = (int16_t)lrintf(v);
        fwrite(&s, 2, 1, f);
    }
    return fclose(f) == 0;
}

// SURVEY.md §8(d) recipe; uniform/normal derived from raw mt19937_64 output
// so the samples do not depend on the C++ library's distribution classes.
void synth_pcm(uint64_t seed, int n, float *out) {
    std::mt19937_64 rng(seed);
    auto uni = [&]() { return (double)(rng() >> 11) * (1.0 / 9007199254740992.0); };
    const double f0 = 100.0 + 200.0 * uni(), f1 = 500.0 + 2500.0 * uni(), am = 2.0 + 4.0 * uni();
    for (int i = 0; i < n; i++) {
        double t = i / 16000.0;
        double u1 = uni(), u2 = uni();
        double g = sqrt(-2.0 * log(u1 > 1e-300 ? u1 : 1e-300)) * cos(2.0 * M_PI * u2);
        double x = 0.25 * sin(2.0 * M_PI * f0 * t) + 0.2 * (0.5 + 0.5 * sin(2.0 * M_PI * am * t)) * sin(2.0 * M_PI * f1 * t) +
                   0.03 * g;
        x = x > 1.0 ? 1.0 : (x < -1.0 ? -1.0 : x);
        int16_t q = (int16_t)lrint(32767.0 * x);
        out[i] = q / 32768.0f;   // as load_wav would return it
    }
}

// ------------------------------------------------------------------ text
static void byte_tables(std::vector<std::string> &b2u, std::vector<int> &cp2b) {
    std::vector<int> cp(256, -1);
    for (int b = 0x21; b <= 0x7e; b++) cp[b] = b;
    for (int b = 0xa1; b <= 0xac; b++) cp[b] = b;
    for (int b = 0xae; b <= 0xff; b++) cp[b] = b;
    int n = 0;
    for (int b = 0; b < 256; b++) if (cp[b] < 0) cp[b] = 256 + n++;
    b2u.assign(256, "");
    cp2b.assign(512, -1);
    for (int b = 0; b < 256; b++) {
        int c = cp[b];
        std::string s;
        if (c < 0x80) s += (char)c;
        else { s += (char)(0xC0 | (c >> 6)); s += (char)(0x80 | (c & 0x3F)); }
        b2u[b] = s;
        cp2b[c] = b;
    }
}

static const std::vector<std::string> &bytes_to_unicode() {
    static const std::vector<std::string> t = [] { std::vector<std::string> a; std::vector<int> b; byte_tables(a, b); return a; }();
    return t;
}
static const std::vector<int> &unicode_to_byte() {
    static const std::vector<int> t = [] { std::vector<std::string> a; std::vector<int> b; byte_tables(a, b); return b; }();
    return t;
}

bool Tokenizer::load(const GGUFFile &f, std::string &err) {
    if (!f.get_str_array("tokenizer.ggml.tokens", vocab_)) { err = "Vocabulary not found in GGUF file"; return false; }
    if (vocab_.empty()) { err = "Empty vocabulary in GGUF file"; return false; }
    tok2id_.clear();
    tok2id_.reserve(vocab_.size());
    for (size_t i = 0; i < vocab_.size(); i++) tok2id_[vocab_[i]] = (int32_t)i;
    std::vector<std::string> merges;
    ranks_.clear();
    if (f.get_str_array("tokenizer.ggml.merges", merges))
        for (size_t i = 0; i < merges.size(); i++) ranks_[merges[i]] = (int)i;
    return true;
}

// src/text_decoder.cpp:985-1067
std::string Tokenizer::decode_token(int32_t id) const {
    if (id < 0 || id >= (int32_t)vocab_.size()) return "";
    const std::string &t = vocab_[id];
    const size_t L = t.size();
    if (L >= 3 && t[0] == '<' && t[1] == '|' && t[L - 1] == '>' && t[L - 2] == '|') return "";
    if (L >= 5 && t.compare(0, 4, "[PAD") == 0) return "";
    const std::vector<int> &cp2b = unicode_to_byte();
    std::string out;
    size_t i = 0;
    while (i < L) {
        unsigned char c = (unsigned char)t[i];
        uint32_t cp;
        size_t len;
        if (c < 0x80) { cp = c; len = 1; }
        else if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; len = 2; }
        else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; len = 3; }
        else if ((c & 0xF8) == 0xF0) { cp = c & 0x07; len = 4; }
        else { out += (char)c; i++; continue; }
        if (i + len > L) { out.append(t, i, std::string::npos); break; }
        for (size_t j = 1; j < len; j++) cp = (cp << 6) | ((unsigned char)t[i + j] & 0x3F);
        i += len;
        if (cp < cp2b.size() && cp2b[cp] >= 0) out += (char)cp2b[cp];
        else if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        } else {
            out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        }
    }
    return out;
}

std::string Tokenizer::decode(const std::vector<int32_t> &ids) const {
    std::string s;
    for (int32_t id : ids) s += decode_token(id);
    return s;
}

static std::vector<std::string> utf8_chars(const std::string &s) {
    std::vector<std::string> out;
    for (size_t i = 0; i < s.size();) {
        unsigned char c = (unsigned char)s[i];
        size_t len = 1;
        if ((c & 0xE0) == 0xC0) len = 2;
        else if ((c & 0xF0) == 0xE0) len = 3;
        else if ((c & 0xF8) == 0xF0) len = 4;
        if (i + len > s.size()) len = 1;
        out.push_back(s.substr(i, len));
        i += len;
    }
    return out;
}

// src/text_decoder.cpp:911-949 + :1077-1103
std::vector<int32_t> Tokenizer::encode(const std::string &text) const {
    std::vector<int32_t> ids;
    std::istringstream iss(text);
    std::string word;
    bool first = true;
    const auto &b2u = bytes_to_unicode();
    while (iss >> word) {
        std::string w = first ? word : " " + word;
        first = false;
        std::string bpe;
        for (unsigned char c : w) bpe += b2u[c];
        std::vector<std::string> sym = utf8_chars(bpe);
        while (sym.size() > 1) {
            int best = INT_MAX;
            size_t pos = 0;
            for (size_t i = 0; i + 1 < sym.size(); i++) {
                auto it = ranks_.find(sym[i] + " " + sym[i + 1]);
                if (it != ranks_.end() && it->second < best) { best = it->second; pos = i; }
            }
            if (best == INT_MAX) break;
            sym[pos] += sym[pos + 1];
            sym.erase(sym.begin() + (long)pos + 1);
        }
        for (auto &s : sym) {
            auto it = tok2id_.find(s);
            if (it != tok2id_.end()) ids.push_back(it->second);
        }
    }
    return ids;
}

std::vector<int32_t> Tokenizer::encode_word(const std::string &word) const {
    std::vector<int32_t> ids;
    const auto &b2u = bytes_to_unicode();
    std::string bpe;
    for (unsigned char c : word) bpe += b2u[c];
    std::vector<std::string> sym = utf8_chars(bpe);
    while (sym.size() > 1) {
        int best = INT_MAX;
        size_t pos = 0;
        for (size_t i = 0; i + 1 < sym.size(); i++) {
            auto it = ranks_.find(sym[i] + " " + sym[i + 1]);
            if (it != ranks_.end() && it->second < best) { best = it->second; pos = i; }
        }
        if (best == INT_MAX) break;
        sym[pos] += sym[pos + 1];
        sym.erase(sym.begin() + (long)pos + 1);
    }
    for (auto &sw : sym) {
        auto it = tok2id_.find(sw);
        if (it != tok2id_.end()) ids.push_back(it->second);
        else fprintf(stderr, "BPE tokenizer: unknown subword token '%s'\n", sw.c_str());
    }
    return ids;
}

// ------------------------------------------------------- forced aligner
static bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

std::vector<std::string> split_words(const std::string &text) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < text.size()) {
        while (i < text.size() && is_ws(text[i])) ++i;
        if (i >= text.size()) break;
        const size_t st = i;
        while (i < text.size() && !is_ws(text[i])) ++i;
        out.push_back(text.substr(st, i - st));
    }
    return out;
}

static size_t u8len(unsigned char c) {
    if ((c & 0x80) == 0) return 1;
    if ((c & 0xE0) == 0xC0) return 2;
    if ((c & 0xF0) == 0xE0) return 3;
    if ((c & 0xF8) == 0xF0) return 4;
    return 1;
}

// first n characters / the rest, by UTF-8 lead bytes (clamped at the end)
static void u8split(const std::string &s, size_t n, std::string &left, std::string &right) {
    size_t b = 0;
    for (size_t c = 0; c < n && b < s.size(); c++) b += u8len((unsigned char)s[b]);
    if (b > s.size()) b = s.size();
    left = s.substr(0, b);
    right = s.substr(b);
}

std::vector<std::string> tokenize_korean(const std::string &text, const std::unordered_map<std::string, int> &dict) {
    std::vector<std::string> out;
    for (const std::string &w : split_words(text)) {
        size_t len = 0;
        for (size_t i = 0; i < w.size(); i += u8len((unsigned char)w[i])) len++;
        if (len <= 2) { out.push_back(w); continue; }
        // the longest dictionary prefix of >= 2 characters wins; with none, the
        // whole word (score ties go to the longer left part)
        float best = -1e9f;
        size_t best_e = 0;
        std::string bl, br;
        for (size_t e = 2; e <= len; e++) {
            std::string l, r;
            u8split(w, e, l, r);
            const float sc = dict.count(l) ? 1.0f : 0.0f;
            if (sc > best || (sc == best && e > best_e)) { best = sc; best_e = e; bl = l; br = r; }
        }
        out.push_back(bl);
        if (!br.empty()) out.push_back(br);
    }
    return out;
}

bool load_korean_dict(const std::string &path, std::unordered_map<std::string, int> &dict) {
    FILE *fp = fopen(path.c_str(), "rb");
    if (!fp) return false;
    dict.clear();
    std::string line;
    int ch;
    auto flush = [&] {
        if (!line.empty() && line.back() == '\r') line.pop_back();   // std::getline keeps a CR; only the first field matters
        if (!line.empty()) {
            const size_t sp = line.find(' ');
            const std::string word = sp == std::string::npos ? line : line.substr(0, sp);
            if (!word.empty()) dict.emplace(word, 1);
        }
        line.clear();
    };
    while ((ch = fgetc(fp)) != EOF) {
        if (ch == '\n') flush();
        else line += (char)ch;
    }
    flush();
    fclose(fp);
    return true;
}

int feat_extract_output_lengths(int n) {
    const int leave = n % 100;
    const int feat = (leave - 1) / 2 + 1;
    return ((feat - 1) / 2 + 1 - 1) / 2 + 1 + (n / 100) * 13;
}

std::vector<int32_t> fix_timestamp_classes(const std::vector<int32_t> &data) {
    const int n = (int)data.size();
    if (n == 0) return {};
    std::vector<int> dp(n, 1), parent(n, -1);
    for (int i = 1; i < n; i++)
        for (int j = 0; j < i; j++)
            if (data[j] <= data[i] && dp[j] + 1 > dp[i]) { dp[i] = dp[j] + 1; parent[i] = j; }
    int max_len = 0, max_idx = 0;
    for (int i = 0; i < n; i++)
        if (dp[i] > max_len) { max_len = dp[i]; max_idx = i; }
    std::vector<bool> normal(n, false);
    for (int i = max_idx; i != -1; i = parent[i]) normal[i] = true;
    std::vector<int32_t> r(data);
    int i = 0;
    while (i < n) {
        if (normal[i]) { ++i; continue; }
        int j = i;
        while (j < n && !normal[j]) ++j;
        const int cnt = j - i;
        int32_t lv = -1, rv = -1;
        for (int k = i - 1; k >= 0; --k) if (normal[k]) { lv = r[k]; break; }
        for (int k = j; k < n; ++k) if (normal[k]) { rv = r[k]; break; }
        if (cnt <= 2) {
            for (int k = i; k < j; ++k) r[k] = lv < 0 ? rv : (rv < 0 ? lv : ((k - (i - 1)) <= (j - k) ? lv : rv));
        } else if (lv >= 0 && rv >= 0) {
            const float step = (float)(rv - lv) / (cnt + 1);
            for (int k = i; k < j; ++k) r[k] = (int32_t)(lv + step * (k - i + 1));
        } else if (lv >= 0) {
            for (int k = i; k < j; ++k) r[k] = lv;
        } else if (rv >= 0) {
            for (int k = i; k < j; ++k) r[k] = rv;
        }
        i = j;
    }
    return r;
}

std::vector<int32_t> build_align_tokens(const Hparams &hp, const std::vector<int32_t> &text_tokens, int n_pads) {
    std::vector<int32_t> t;
    t.reserve(text_tokens.size() + n_pads + 2);
    t.push_back(hp.audio_start_id);
    for (int i = 0; i < n_pads; i++) t.push_back(hp.audio_pad_id);
    t.push_back(hp.audio_end_id);
    t.insert(t.end(), text_tokens.begin(), text_tokens.end());
    return t;
}

// ---------------------------------------------------------------- prompt
std::vector<int32_t> build_prompt(const Hparams &hp, int n_audio, const std::vector<int32_t> &sys, int *audio_pos) {
    const int32_t im_start = 151644, im_end = 151645, sys_tok = 8948, user = 872, asst = 77091, nl = 198;
    std::vector<int32_t> t = {im_start, sys_tok, nl};
    t.insert(t.end(), sys.begin(), sys.end());
    t.insert(t.end(), {im_end, nl, im_start, user, nl, hp.audio_start_id});
    if (audio_pos) *audio_pos = n_audio > 0 ? (int)t.size() : -1;
    for (int i = 0; i < n_audio; i++) t.push_back(hp.audio_pad_id);
    t.insert(t.end(), {hp.audio_end_id, im_end, nl, im_start, asst, nl});
    return t;
}

// ------------------------------------------------------- synthetic GGUF
static inline uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline float gauss(uint64_t seed, uint64_t tid, uint64_t i) {
    uint64_t a = splitmix(seed ^ splitmix(tid * 0x100000001B3ull + 0x12345) ^ (i * 2 + 0));
    uint64_t b = splitmix(a ^ 0xD1B54A32D192ED03ull);
    double u1 = ((a >> 11) + 1) * (1.0 / 9007199254740993.0), u2 = (b >> 11) * (1.0 / 9007199254740992.0);
    return (float)(sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2));
}

struct SynTensor { std::string name; std::vector<int64_t> ne; int kind; float scale; };  // kind 0 matrix,1 norm,2 bias,3 embd

bool write_synthetic_gguf(const std::string &path, const std::string &config, uint64_t seed, int wtype, std::string &err) {
    Hparams hp;
    // "full"/"tiny": Qwen3-ASR; "aligner"/"aligner-tiny": Qwen3-ForcedAligner
    // (src/forced_aligner.h:36-73: 24 x 1024 encoder, 16 heads, ffn 4096,
    // vocab 152064, 5000-class head)
    const bool al = config == "aligner" || config == "aligner-tiny";
    const bool tiny = config == "tiny" || config == "aligner-tiny";
    if (!tiny && config != "full" && config != "aligner") {
        err = "unknown synthetic config: " + config;
        return false;
    }
    if (al) {
        hp.aligner = true;
        hp.classify_num = 5000;
        if (!tiny) { hp.enc_layers = 24; hp.d_model = 1024; hp.enc_heads = 16; hp.enc_ffn = 4096; hp.vocab = 152064; }
    }
    if (tiny) {
        hp.enc_layers = 2; hp.d_model = 256; hp.enc_heads = 4; hp.enc_ffn = 512; hp.conv_ch = 96;
        hp.hidden = 256; hp.dec_layers = 2; hp.n_head = 4; hp.n_kv_head = 2; hp.head_dim = 128; hp.dec_ffn = 512;
    }
    if (wtype != 1 && wtype != 8) { err = "wtype must be 1 (f16) or 8 (q8_0)"; return false; }
    GGUFWriter w;
    w.add_str("general.architecture", "qwen3-asr");
    w.add_str("general.name", al ? (tiny ? "Qwen3-ForcedAligner-synthetic-tiny" : "Qwen3-ForcedAligner-0.6B-synthetic")
                                 : (tiny ? "Qwen3-ASR-synthetic-tiny" : "Qwen3-ASR-0.6B-synthetic"));
    w.add_u32("general.alignment", 32);
    w.add_u32("qwen3-asr.block_count", hp.dec_layers);
    w.add_u32("qwen3-asr.embedding_length", hp.hidden);
    w.add_u32("qwen3-asr.feed_forward_length", hp.dec_ffn);
    w.add_u32("qwen3-asr.attention.head_count", hp.n_head);
    w.add_u32("qwen3-asr.attention.head_count_kv", hp.n_kv_head);
    w.add_u32("qwen3-asr.attention.key_length", hp.head_dim);
    w.add_u32("qwen3-asr.attention.value_length", hp.head_dim);
    w.add_f32("qwen3-asr.rope.freq_base", hp.rope_theta);
    w.add_f32("qwen3-asr.attention.layer_norm_rms_epsilon", hp.rms_eps);
    w.add_u32("qwen3-asr.vocab_size", hp.vocab);
    w.add_u32("qwen3-asr.audio.encoder.layer_count", hp.enc_layers);
    w.add_u32("qwen3-asr.audio.encoder.embedding_length", hp.d_model);
    w.add_u32("qwen3-asr.audio.encoder.attention.head_count", hp.enc_heads);
    w.add_u32("qwen3-asr.audio.encoder.feed_forward_length", hp.enc_ffn);
    w.add_u32("qwen3-asr.audio.num_mel_bins", hp.n_mel);
    w.add_u32("qwen3-asr.audio.conv_channels", hp.conv_ch);
    w.add_u32("qwen3-asr.audio.start_token_id", hp.audio_start_id);
    w.add_u32("qwen3-asr.audio.end_token_id", hp.audio_end_id);
    w.add_u32("qwen3-asr.audio.pad_token_id", hp.audio_pad_id);
    if (al) {   // scripts/convert_hf_to_gguf.py:454-458
        w.add_u32("qwen3-asr.classify_num", hp.classify_num);
        w.add_u32("qwen3-asr.timestamp_token_id", hp.timestamp_id);
        w.add_u32("qwen3-asr.timestamp_segment_time", hp.ts_segment_ms);
    }
    if (tiny && !al) {   // the reference's own encoder keys (src/gguf_loader.cpp:69-85)
        w.add_u32("audio.encoder_layers", hp.enc_layers);
        w.add_u32("audio.d_model", hp.d_model);
        w.add_u32("audio.attention_heads", hp.enc_heads);
        w.add_u32("audio.ffn_dim", hp.enc_ffn);
        w.add_u32("audio.conv_channels", hp.conv_ch);
        w.add_u32("text.hidden_size", hp.hidden);
    }
    // synthetic byte-level vocabulary (ids 0..255 are the GPT-2 byte symbols)
    std::vector<std::string> toks(hp.vocab);
    const auto &b2u = bytes_to_unicode();
    std::vector<int> order;
    for (int b = 0x21; b <= 0x7e; b++) order.push_back(b);
    for (int b = 0xa1; b <= 0xac; b++) order.push_back(b);
    for (int b = 0xae; b <= 0xff; b++) order.push_back(b);
    for (int b = 0; b < 256; b++) if (!((b >= 0x21 && b <= 0x7e) || (b >= 0xa1 && b <= 0xac) || (b >= 0xae && b <= 0xff))) order.push_back(b);
    for (int i = 0; i < 256; i++) toks[i] = b2u[order[i]];
    std::vector<std::string> merges;
    for (int i = 256; i < hp.vocab; i++) {
        if (i < 151643) {
            int v = i - 256;
            std::string s = (v & 1) ? b2u[' '] : "";
            int n = v / 2;
            do { s += (char)('a' + n % 26); n /= 26; } while (n > 0);
            toks[i] = s;
            if (s.size() == 2 && !(v & 1)) merges.push_back(std::string(1, s[0]) + " " + s[1]);
        } else {
            toks[i] = "<|extra_" + std::to_string(i - 151643) + "|>";
        }
    }
    toks[151643] = "<|endoftext|>";
    toks[151644] = "<|im_start|>";
    toks[151645] = "<|im_end|>";
    toks[hp.audio_start_id] = "<|audio_start|>";
    toks[hp.audio_end_id] = "<|audio_end|>";
    toks[hp.audio_pad_id] = "<|audio_pad|>";
    for (int i = 151677; i < hp.vocab; i++) toks[i] = "[PAD" + std::to_string(i) + "]";
    if (al) toks[hp.timestamp_id] = "<timestamp>";
    w.add_str("tokenizer.ggml.model", "gpt2");
    w.add_str_array("tokenizer.ggml.tokens", toks);
    w.add_str_array("tokenizer.ggml.merges", merges);

    // tensors: names scripts/convert_hf_to_gguf.py:50-120; dtypes :254-311
    std::vector<SynTensor> ts;
    const int C = hp.conv_ch, D = hp.d_model, FF = hp.enc_ffn, H = hp.hidden;
    auto mat = [&](const std::string &n, std::vector<int64_t> ne) {
        int64_t fan = ne[0];
        if (ne.size() == 4) fan = ne[0] * ne[1] * ne[2];
        ts.push_back({n, ne, 0, 1.0f / sqrtf((float)fan)});
    };
    auto vec = [&](const std::string &n, int64_t len, int kind) { ts.push_back({n, {len}, kind, kind == 1 ? 0.1f : 0.02f}); };
    mat("audio.encoder.conv1.weight", {3, 3, 1, C});
    vec("audio.encoder.conv1.bias", C, 2);
    mat("audio.encoder.conv2.weight", {3, 3, C, C});
    vec("audio.encoder.conv2.bias", C, 2);
    mat("audio.encoder.conv3.weight", {3, 3, C, C});
    vec("audio.encoder.conv3.bias", C, 2);
    mat("audio.encoder.conv_out.weight", {(int64_t)C * 16, D});
    for (int l = 0; l < hp.enc_layers; l++) {
        std::string p = "audio.encoder.blk." + std::to_string(l) + ".";
        for (const char *nm : {"attn_q", "attn_k", "attn_v", "attn_out"}) {
            mat(p + nm + ".weight", {D, D});
            vec(p + nm + ".bias", D, 2);
        }
        vec(p + "attn_norm.weight", D, 1);
        vec(p + "attn_norm.bias", D, 2);
        mat(p + "ffn_up.weight", {D, FF});
        vec(p + "ffn_up.bias", FF, 2);
        mat(p + "ffn_down.weight", {FF, D});
        vec(p + "ffn_down.bias", D, 2);
        vec(p + "ffn_norm.weight", D, 1);
        vec(p + "ffn_norm.bias", D, 2);
    }
    vec("audio.encoder.ln_post.weight", D, 1);
    vec("audio.encoder.ln_post.bias", D, 2);
    mat("audio.encoder.proj1.weight", {D, D});
    vec("audio.encoder.proj1.bias", D, 2);
    mat("audio.encoder.proj2.weight", {D, H});
    vec("audio.encoder.proj2.bias", H, 2);
    ts.push_back({"token_embd.weight", {H, hp.vocab}, 3, 4.0f / sqrtf((float)H)});
    vec("output_norm.weight", H, 1);
    // aligner classification head: F16 in every file type (convert_hf_to_gguf.py:240-241)
    if (al) ts.push_back({"output.weight", {H, hp.classify_num}, 3, 4.0f / sqrtf((float)H)});
    const int QD = hp.n_head * hp.head_dim, KD = hp.n_kv_head * hp.head_dim;
    for (int l = 0; l < hp.dec_layers; l++) {
        std::string p = "blk." + std::to_string(l) + ".";
        vec(p + "attn_norm.weight", H, 1);
        mat(p + "attn_q.weight", {H, QD});
        mat(p + "attn_k.weight", {H, KD});
        mat(p + "attn_v.weight", {H, KD});
        mat(p + "attn_output.weight", {QD, H});
        vec(p + "attn_q_norm.weight", hp.head_dim, 1);
        vec(p + "attn_k_norm.weight", hp.head_dim, 1);
        vec(p + "ffn_norm.weight", H, 1);
        mat(p + "ffn_gate.weight", {H, hp.dec_ffn});
        mat(p + "ffn_up.weight", {H, hp.dec_ffn});
        mat(p + "ffn_down.weight", {hp.dec_ffn, H});
    }
    std::vector<uint32_t> types(ts.size());
    for (size_t i = 0; i < ts.size(); i++) {
        const SynTensor &t = ts[i];
        uint32_t ty = t.ne.size() == 1 ? DT_F32 : DT_F16;
        // q8_0: linear weights only; embeddings/conv kernels stay F16
        // (convert_hf_to_gguf.py:229-252, 293-308)
        if (ty == DT_F16 && wtype == DT_Q8_0 && t.kind == 0 && t.ne.size() == 2 && t.ne[0] % 32 == 0) ty = DT_Q8_0;
        types[i] = ty;
        w.add_tensor(t.name, ty, t.ne);
    }
    bool ok = w.write(path, [&](size_t i, uint8_t *dst, size_t nbytes) {
        const SynTensor &t = ts[i];
        int64_t n = 1;
        for (auto v : t.ne) n *= v;
        const uint64_t tid = i + 1;
        if (types[i] == DT_F32) {
            float *o = (float *)dst;
            #pragma omp parallel for schedule(static)
            for (int64_t j = 0; j < n; j++) {
                float g = gauss(seed, tid, (uint64_t)j);
                o[j] = t.kind == 1 ? 1.0f + t.scale * g : t.scale * g;
            }
        } else if (types[i] == DT_F16) {
            uint16_t *o = (uint16_t *)dst;
            #pragma omp parallel for schedule(static)
            for (int64_t j = 0; j < n; j++) o[j] = f32_to_f16(t.scale * gauss(seed, tid, (uint64_t)j));
        } else {   // Q8_0 block: fp16 d = amax/127, q = round(x/d) (ggml quantize_row_q8_0_ref)
            const int64_t nb = n / 32;
            #pragma omp parallel for schedule(static)
            for (int64_t b = 0; b < nb; b++) {
                float x[32], amax = 0.0f;
                for (int j = 0; j < 32; j++) {
                    x[j] = t.scale * gauss(seed, tid, (uint64_t)(b * 32 + j));
                    amax = fmaxf(amax, fabsf(x[j]));
                }
                const float d = amax / 127.0f, id = d ? 1.0f / d : 0.0f;
                uint8_t *blk = dst + b * 34;
                uint16_t dh = f32_to_f16(d);
                memcpy(blk, &dh, 2);
                for (int j = 0; j < 32; j++) blk[2 + j] = (uint8_t)(int8_t)roundf(x[j] * id);
            }
        }
        (void)nbytes;
        return true;
    });
    if (!ok) err = w.error;
    return ok;
}

}  // namespace qasr
