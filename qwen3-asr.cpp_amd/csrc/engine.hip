// engine.hip -- C-ABI implementation (include/qasr_capi.h): device weight
// arena, per-context buffers, and the hot path
//   PCM -> mel -> conv front-end -> encoder -> prompt + splice -> prefill ->
//   greedy decode (HIP-graph replayed step) -> token ids
// restating Qwen3ASR::transcribe_internal (src/qwen3_asr.cpp:81-149) on HIP.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <map>
#include <vector>

#include "../../include/qasr_capi.h"
#include "../host/gguf.h"
#include "../host/qasr_host.h"
#include "dev_common.h"
#include "kernels.h"

using namespace qasr;

static constexpr int kStampRec = 2 * STAMP_ENDS;   // u64 per probed launch record (dev_common.h stamp_start/end)

static thread_local std::string g_err;

static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

// a GEMM / GEMV launch that found no kernel for its (mode, epilogue) pair
// (gemm.hip note_declined) fails the stage that issued it
static int declined_check(const char *stage) {
    std::string msg;
    if (qasr::take_declined(&msg)) return fail(QASR_ERR_STATE, std::string(stage) + ": " + msg);
    return 0;
}

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) return fail(QASR_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------ model
// Linear weights are fp16 [N][K] (F16 files) or int8 [N][K] quants with fp16
// block scales *_d [N][K/32] (Q8_0 files: block_q8_0 split in two arrays).
struct EncLayer {
    uint16_t *wqkv, *wo, *w1, *w2;
    uint16_t *wqkv_d = nullptr, *wo_d = nullptr, *w1_d = nullptr, *w2_d = nullptr;
    float *bqkv, *bo, *b1, *b2, *ln1_w, *ln1_b, *ln2_w, *ln2_b;
};
struct DecLayer {
    float *attn_norm, *q_norm, *k_norm, *ffn_norm;
    uint16_t *wqkv, *wo, *wgu, *wd;
    uint16_t *wqkv_d = nullptr, *wo_d = nullptr, *wgu_d = nullptr, *wd_d = nullptr;
};

struct qasr_model {
    Hparams hp;
    int device = 0;
    Tokenizer tok;
    char *arena = nullptr;
    size_t arena_bytes = 0;
    uint16_t *conv1_w, *conv2_w, *conv3_w, *conv_out_w, *proj1_w, *proj2_w, *embd;
    uint16_t *conv_out_d = nullptr, *proj1_d = nullptr, *proj2_d = nullptr;
    bool q8 = false;   // linear weights are Q8_0 (scripts/convert_hf_to_gguf.py:230-308)
    uint16_t *cls_w = nullptr;   // aligner: classify head [cls_rows][hidden] fp16, rows >= classify_num zero
    int cls_rows = 0;
    std::unordered_map<std::string, int> ko_dict;   // aligner: Korean word list (src/forced_aligner.cpp:1543-1562)
    float *conv1_b, *conv2_b, *conv3_b, *ln_post_w, *ln_post_b, *proj1_b, *proj2_b, *out_norm;
    std::vector<EncLayer> enc;
    std::vector<DecLayer> dec;
    uint16_t *gelu;
    float *pe, *filters;
    double2 *tw;
    double *hann;
    ~qasr_model() {
        if (arena && device >= 0) {
            (void)hipSetDevice(device);
            (void)hipFree(arena);
        }
    }
};

// --------------------------------------------------------------- context
struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    template <class T> T *as() const { return (T *)p; }
};

struct qasr_ctx {
    qasr_model *m = nullptr;
    int max_batch = 0, max_ctx = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev[8] = {};
    uint16_t *kc = nullptr, *vc = nullptr;
    uint16_t *vt = nullptr;        // V^T cache (kernels.h vt_ctx): the exact decode attention's V
    float *rope = nullptr;
    std::vector<DevBuf> owned;     // everything hipMalloc'ed by the context
    // grow-on-demand scratch
    DevBuf pcm, spcm, mel, meltmp, melmax, melclips, melblocks;   // (spcm: qasr_run_stream's host clips)
    DevBuf chunks, rs1, rs2, rs3, pepos, act1, act2, act3;
    DevBuf pebig;                  // encode_no_chunk: sinusoidal PE over a whole clip's frames
    int pebig_rows = 0;
    DevBuf ex, exh, eqkv, eatt, eff, feats, segs;
    DevBuf px, pxh, pqkv, pq, patt, pact, prow, plast, pids, pxl;
    DevBuf pq32, pk32;             // ForcedAligner prefill: fp32 Q / K rows
    DevBuf ats, atx, aam;          // aligner: timestamp-row indices, their normed rows, argmax keys
    DevBuf exp_, gidx;             // aligner batches: conv_out over every padded chunk row, the valid rows' indices
    DevBuf q8a, q8d, x32;          // Q8_0 models: quantised activations (int8 + scales), fp32 layer inputs
    float *d_att32 = nullptr, *d_act32 = nullptr;   // Q8_0 decode: fp32 attention output / SwiGLU output
    int8_t *d_q8a = nullptr; float *d_q8d = nullptr, *d_x32 = nullptr;   // Q8_0 batched (B > 8) decode, graph-fixed
    int8_t *d_q8n = nullptr; float *d_q8nd = nullptr;   // ... the RMS-normed layer inputs (QKV, gate/up), quantised
    // fixed decode state (sized by max_batch)
    int32_t *d_tok = nullptr, *d_hist = nullptr;
    int *d_pos = nullptr, *d_nkv = nullptr, *d_slot = nullptr, *d_step = nullptr;
    float *d_x = nullptr, *d_qkv = nullptr, *d_part = nullptr, *d_logits = nullptr;
    float *d_scores = nullptr;     // exact decode attention: [B][n_head][max_ctx] scaled scores
    unsigned int *d_counter = nullptr, *d_done = nullptr;
    unsigned int *d_qcnt = nullptr;   // fused batch-1 QKV + attention: QKV-block arrivals per kv group
    unsigned long long *d_gran = nullptr;   // ... or its outputs as tagged granules (zeroed by every prefill)
    unsigned long long *d_sgran = nullptr;  // ... exact attention: the splits' scores as granules [n_head][max_ctx] (zeroed likewise)
    bool qkv_in_gran = false;               // the captured step's last layer hands its QKV over in granules
    unsigned int *d_attdone = nullptr;   // fused batch-1 o-proj: combiner arrivals, [layer][8 replicas][16]
    unsigned int *d_ffncnt = nullptr;    // fused batch-1 FFN: [layer][gate/up arrivals, o-proj arrivals][32 shards][16]
    uint16_t *d_q = nullptr, *d_att = nullptr, *d_act = nullptr, *d_xh = nullptr;
    unsigned long long *d_amax = nullptr;
    int max_splits = 0, hist_cap = 0;
    // pinned host staging for small per-call tables (reset at each top-level call)
    char *pin = nullptr;
    size_t pin_cap = 0, pin_used = 0;
    std::vector<int32_t> sys_ids;
    // staged audio
    std::vector<int> staged_n;
    std::vector<long> staged_off;
    bool eager = false;            // QASR_NO_GRAPH=1: launch the decode step eagerly (profilers)
    int dev_skip = 0;              // QASR_DEV_SKIP bitmask (-DQASR_DIAG_SKIP builds only): omits decode kernels
    FuseCfg fuse;                  // batch-1 fused launches: switches, delays, co-residency of this device
    unsigned int *d_err = nullptr; // sticky device error word of the fused launches (DevErr bits)
    int dbg_layers = 0;            // diagnostic: decode steps run only the first n decoder layers (0 = all)
    // --profile (src/timing.h QWEN3_TIMER sections): per-section device time from
    // HIP events, accumulated over calls until qasr_set_profile resets it
    bool profile_on = false;
    std::map<std::string, std::pair<double, long>> prof;   // section -> (total ms, calls)
    std::vector<hipEvent_t> step_ev;                       // per decode step, profile only
    // per-token callback (src/qwen3_asr.cpp:264-291): called synchronously
    // after every greedy step of qasr_run, in order, for every live sequence
    void (*tok_cb)(void *user, int seq, int n_generated, int32_t token) = nullptr;
    void *tok_cb_user = nullptr;
    // QASR_DEV_TRACE=<file>: per-block timestamps of one decode layer's kernels
    // (layer QASR_DEV_TRACE_LAYER, default 10) of the last step, dumped by qasr_run
    std::string trace_path;
    int trace_layer = 10;
    unsigned long long *d_trace = nullptr;   // [6 kernels][4096 blocks][8]
    // kernel probe: HIP-event timing of one decode-step kernel inside qasr_run
    int probe = 0;                 // 0 off, 1 LM head, 2 layer QKV + attention, 3 layer FFN
    int probe_layer = 14;          // decoder layer whose groups probes 2 / 3 time
    int probe_stride = 1;          // probe decode steps k with k % probe_stride == 0 (the others replay the whole-step
                                   // graph: the probed step's split graphs and eager group cost ~3 % of a step)
    bool probe_o_fused = false;    // the probed layer's o-projection runs inside the QKV launch
    int last_fmode = 0, last_fx = 0;   // the last emitted decode step, layer 0: fused launch mode (0 separate, 1 QKV +
                                       // attention, 2 + o-proj) and whether its attention was the chain role (options
                                       // "fused_mode" / "fused_exact", read-only)
    int last_attn = 0;             // the same step's decode attention launches (option "attn_path", read-only): 0 split-K
                                   // fp32, 1 chain role of the fused launch, 2 scores + chain in one launch per sequence
                                   // (decode_attn_seq_kernel), 3 separate scores and chain kernels
    double probe_ms = 0.0, probe_bytes = 0.0, probe_dev_ms = 0.0;
    long probe_dev_n = 0;
    unsigned long long *d_pstamp = nullptr;   // per decode step: [32 min-starts | 32 max-ends] of the probed launches
    unsigned long long *cur_stamp = nullptr;  // record of the group being emitted (probe only)
    long probe_n = 0;
    std::vector<int> run_P;        // prompt lengths of the current qasr_run (decode step k: n_kv = P_b + k + 1)
    std::vector<hipEvent_t> pev;
    // decode graphs, one set per attention split-grid bucket (the grid must
    // cover the longest sequence's context: it grows by 64 keys per split)
    struct StepGraphs { hipGraphExec_t full = nullptr, pre = nullptr, post = nullptr; };
    std::map<int, StepGraphs> graphs;   // key: batch * 65536 + split bucket
    int graph_B = -1;
    bool graph_logits = false;
    int graph_base = 0;            // max prompt length of the current run: step k feeds position base + k
    int graph_probe_group = -1;    // launch group timed between events (pre/post graphs split around it)
    void drop_graphs() {
        for (auto &kv : graphs) {
            if (kv.second.full) (void)hipGraphExecDestroy(kv.second.full);
            if (kv.second.pre) (void)hipGraphExecDestroy(kv.second.pre);
            if (kv.second.post) (void)hipGraphExecDestroy(kv.second.post);
        }
        graphs.clear();
    }
    ~qasr_ctx() {
        (void)hipSetDevice(m->device);
        drop_graphs();
        for (auto &e : pev) (void)hipEventDestroy(e);
        for (auto &e : step_ev) (void)hipEventDestroy(e);
        for (auto &b : owned) (void)hipFree(b.p);
        for (auto &e : ev) if (e) (void)hipEventDestroy(e);
        if (pin) (void)hipHostFree(pin);
        if (st) (void)hipStreamDestroy(st);
    }
};

// per-context options of the fused batch-1 launches: name (qasr_ctx_set_option),
// environment default, field
struct FuseOption {
    const char *name, *env;
    int FuseCfg::*field;
};
static const std::vector<FuseOption> &fuse_options() {
    static const std::vector<FuseOption> v = {
        {"fuse_ffn", "QASR_FUSE_FFN", &FuseCfg::ffn},          {"fuse_qkv", "QASR_FUSE_QKV", &FuseCfg::qkv},
        {"fuse_o", "QASR_FUSE_O", &FuseCfg::o},
        {"ffn_delay", "QASR_FFN_DELAY", &FuseCfg::ffn_delay},
        {"ffn_wdelay", "QASR_FFN_WDELAY", &FuseCfg::ffn_wdelay}, {"qkv_delay", "QASR_FUSE_DELAY", &FuseCfg::qkv_delay},
        {"o_delay", "QASR_FUSE_ODELAY", &FuseCfg::o_delay},    {"att_spl1", "QASR_ATT_SPL1", &FuseCfg::spl1},
        {"poll_limit", "QASR_POLL_LIMIT", &FuseCfg::poll_limit}, {"handoff_fence", "QASR_HANDOFF_FENCE", &FuseCfg::fence},
        {"fa_exact_prefill", "QASR_FA_EXACT_PREFILL", &FuseCfg::fa_exact_prefill},
        {"enc_attn_f32", "QASR_ENC_ATTN_F32", &FuseCfg::enc_attn_f32},
        {"gemm_regs", "QASR_GEMM_REGS", &FuseCfg::gemm_regs},
        {"gran", "QASR_GRAN", &FuseCfg::gran},
        {"fa_exact_decode", "QASR_FA_EXACT_DECODE", &FuseCfg::fa_exact_decode},
        {"fx_vpf", "QASR_FX_VPF", &FuseCfg::fx_vpf},
        {"att_stream", "QASR_ATT_STREAM", &FuseCfg::att_stream},
        {"skinny", "QASR_SKINNY", &FuseCfg::skinny},
        {"att_spl", "QASR_ATT_SPL", &FuseCfg::att_spl},
        {"kv_nt", "QASR_KV_NT", &FuseCfg::kv_nt},
        {"lmh", "QASR_LMH", &FuseCfg::lmh},
        {"fx_seq", "QASR_FX_SEQ", &FuseCfg::fx_seq},
        {"skinny_inf", "QASR_SKINNY_INF", &FuseCfg::skinny_inf},
        {"skinny_wdef", "QASR_SKINNY_WDEF", &FuseCfg::skinny_wdef},
        {"refill_group", "QASR_REFILL_GROUP", &FuseCfg::refill_group},
        {"live_prefix", "QASR_LIVE_PREFIX", &FuseCfg::live_prefix},
        {"staged_wrap", "QASR_STAGED_WRAP", &FuseCfg::staged_wrap},
        {"poison_scratch", "QASR_POISON_SCRATCH", &FuseCfg::poison},
    };
    return v;
}

// encoder / prefill GEMMs with the context's tile option
static void launch_gemm_c(qasr_ctx *c, int amode, int epi, GemmArgs g, hipStream_t s) {
    g.regs_staged = c->fuse.gemm_regs;
    launch_gemm(amode, epi, g, s);
}

// every arrival counter of the fused launches back to rest (zero), on the
// context stream: after an option change and after a wait that gave up
static int reset_counters(qasr_ctx *c) {
    const Hparams &hp = c->m->hp;
    HIPCHK(hipMemsetAsync(c->d_ffncnt, 0, (size_t)hp.dec_layers * 1024 * 4, c->st));
    HIPCHK(hipMemsetAsync(c->d_qcnt, 0, (size_t)hp.n_kv_head * 8 * 16 * 4, c->st));
    HIPCHK(hipMemsetAsync(c->d_attdone, 0, (size_t)hp.dec_layers * 128 * 4, c->st));
    HIPCHK(hipMemsetAsync(c->d_counter, 0, (size_t)c->max_batch * hp.n_kv_head * 4, c->st));
    HIPCHK(hipMemsetAsync(c->d_done, 0, 4, c->st));
    HIPCHK(hipMemsetAsync(c->d_amax, 0, (size_t)c->max_batch * 8, c->st));
    return 0;
}

// the fused launches' sticky device error word: read (and cleared) after every
// call that ran decode steps; a bounded wait that ran out is a device error
static int check_dev_err(qasr_ctx *c) {
    unsigned e = 0;
    HIPCHK(hipMemcpyAsync(&e, c->d_err, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (!e) return 0;
    // a wait that gave up can leave late arrivals in the counters: back to rest
    HIPCHK(hipMemsetAsync(c->d_err, 0, 4, c->st));
    const int rc = reset_counters(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->st));
    std::string what;
    if (e & DEVERR_QKV_WAIT) what += " attention<-QKV";
    if (e & DEVERR_O_WAIT) what += " o-proj<-attention";
    if (e & DEVERR_FFN_WAIT) what += " down<-gate/up";
    if (e & DEVERR_SCORE_WAIT) what += " chain<-scores";
    return fail(QASR_ERR_DEVICE, "fused decode launch: an in-launch wait timed out (" + what.substr(1) +
                                     "); outputs of this call are invalid (another process or context sharing the GPU?)");
}

// The batch-1 fused launches assume the whole GPU is theirs (every workgroup
// of a launch co-resident: a role waits on another role in-launch).  Calls
// that can take them hold their device's lock, so contexts driven from
// several host threads on one GPU run those calls one at a time instead of
// sharing the CUs (a GPU shared with another PROCESS is not covered: a wait
// that runs out then fails the call with QASR_ERR_DEVICE; QASR_FUSE_*=0 or
// qasr_ctx_set_option turns the fused launches off).
static std::mutex &device_lock(int device) {
    static std::mutex m[64];
    return m[(unsigned)device % 64];
}
// decode attention with ggml's fp16 V accumulation (fa_exact.hip)?
static bool exact_decode(const qasr_ctx *c) {
    return c->fuse.fa_exact_decode != 0;
}
// V^T cache elements of one layer
static size_t layer_vt(const qasr_ctx *c) {
    return (size_t)c->max_batch * c->m->hp.n_kv_head * 128 * vt_ctx(c->max_ctx);
}
static bool takes_fused(const qasr_ctx *c, int B) {
    return B == 1 && !c->m->q8 && (c->fuse.ffn || c->fuse.qkv);
}

// a roctx range for the lifetime of the object (rocprofv3 --marker-trace)
struct RoctxRange {
    explicit RoctxRange(const char *name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange &) = delete;
    RoctxRange &operator=(const RoctxRange &) = delete;
};

static int dev_alloc(qasr_ctx *c, void **p, size_t bytes) {
    HIPCHK(hipMalloc(p, bytes ? bytes : 256));
    c->owned.push_back({*p, bytes});
    return 0;
}

// grow a scratch buffer (contents are not preserved)
static int ensure(qasr_ctx *c, DevBuf &b, size_t bytes) {
    if (b.n >= bytes && b.p) return 0;
    if (b.p) {
        HIPCHK(hipStreamSynchronize(c->st));
        for (auto it = c->owned.begin(); it != c->owned.end(); ++it)
            if (it->p == b.p) { c->owned.erase(it); break; }
        HIPCHK(hipFree(b.p));
        b.p = nullptr;
    }
    size_t n = std::max<size_t>(bytes + bytes / 4, 4096);
    HIPCHK(hipMalloc(&b.p, n));
    b.n = n;
    c->owned.push_back({b.p, n});
    if (c->fuse.poison) HIPCHK(hipMemsetAsync(b.p, 0xFF, n, c->st));
    return 0;
}

// Small per-call tables go through a pinned staging area so the async copy
// never reads a host vector that has gone out of scope.
template <class T>
static int upload(qasr_ctx *c, DevBuf &b, const std::vector<T> &v) {
    const size_t bytes = v.size() * sizeof(T);
    int rc = ensure(c, b, bytes);
    if (rc || !bytes) return rc;
    const size_t need = (bytes + 255) / 256 * 256;
    if (c->pin_used + need > c->pin_cap) {
        HIPCHK(hipStreamSynchronize(c->st));   // every earlier staged copy has landed
        c->pin_used = 0;
        if (need > c->pin_cap) {
            if (c->pin) HIPCHK(hipHostFree(c->pin));
            c->pin_cap = std::max<size_t>(need * 2, 1 << 20);
            HIPCHK(hipHostMalloc((void **)&c->pin, c->pin_cap, hipHostMallocDefault));
        }
    }
    char *h = c->pin + c->pin_used;
    c->pin_used += need;
    memcpy(h, v.data(), bytes);
    HIPCHK(hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, c->st));
    return 0;
}

// ----------------------------------------------------------------- errors
// A Q8_0 linear layer: quantise the activation rows (fp32 a32 or fp16 a16,
// optional conv_out gather) into c->q8a / c->q8d, then the int8 block GEMM.
// g carries M, N, K and the epilogue.
static void gemm_q8(qasr_ctx *c, int epi, GemmArgs g, const float *a32, const uint16_t *a16, int lda, int gather_C,
                    const uint16_t *W, const uint16_t *Wd, hipStream_t s, int8_t *qa = nullptr, float *qd = nullptr,
                    bool decode = false) {
    if (!qa) { qa = c->q8a.as<int8_t>(); qd = c->q8d.as<float>(); }
    launch_quantize_q8(a32, a16, lda, g.M, g.K, gather_C, qa, qd, s);
    g.Aq = qa; g.lda = g.K; g.Ad = qd; g.ldad = g.K / 32;
    g.Wq = (const int8_t *)W; g.ldw = g.K; g.Wd = Wd;
    g.no_skinny = !c->fuse.skinny;
    g.skinny_inflight = c->fuse.skinny_inf;
    if (decode && launch_gemm_skinny_q8(epi, g, s)) return;
    launch_gemm_q8(epi, g, s);
}

// decode batches: activations already quantised into d_q8a / d_q8d by the
// producing kernel (rmsnorm_q8, the attention combiner)
static void gemm_q8_pre(qasr_ctx *c, int epi, GemmArgs g, const uint16_t *W, const uint16_t *Wd, hipStream_t s,
                        const int8_t *qa = nullptr, const float *qd = nullptr) {
    g.Aq = qa ? qa : c->d_q8a; g.lda = g.K; g.Ad = qa ? qd : c->d_q8d; g.ldad = g.K / 32;
    g.Wq = (const int8_t *)W; g.ldw = g.K; g.Wd = Wd;
    g.no_skinny = !c->fuse.skinny;
    g.skinny_inflight = c->fuse.skinny_inf;
    if (launch_gemm_skinny_q8(epi, g, s)) return;
    launch_gemm_q8(epi, g, s);
}

// decode batches: SwiGLU gate/up with the output quantised to Q8_0 (q / d, row
// length N / 2) in the skinny GEMM's epilogue; false (nothing launched) where
// the skinny GEMM declines the shape or is switched off
static bool gemm_q8_pre_swiglu_q8(qasr_ctx *c, GemmArgs g, const uint16_t *W, const uint16_t *Wd, hipStream_t s, const int8_t *qa,
                                  const float *qd, int8_t *q, float *d) {
    g.Aq = qa; g.lda = g.K; g.Ad = qd; g.ldad = g.K / 32;
    g.Wq = (const int8_t *)W; g.ldw = g.K; g.Wd = Wd;
    g.no_skinny = !c->fuse.skinny;
    g.skinny_inflight = c->fuse.skinny_inf;
    g.out_q = q; g.out_d = d; g.ldoq = g.N / 2;
    return launch_gemm_skinny_q8(EPI_SWIGLU_Q8, g, s);
}

static int ensure_q8(qasr_ctx *c, size_t rows, size_t kmax, size_t x32_cols) {
    int rc;
    if ((rc = ensure(c, c->q8a, rows * kmax)) || (rc = ensure(c, c->q8d, rows * (kmax / 32) * 4)) ||
        (rc = ensure(c, c->x32, rows * x32_cols * 4)))
        return rc;
    return 0;
}

extern "C" const char *qasr_last_error(void) { return g_err.c_str(); }
extern "C" const char *qasr_version(void) { return "qasr-mi355x 0.1.0 (gfx950)"; }
extern "C" int qasr_device_count(int *n) {
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
    if (n) *n = k;
    return 0;
}

extern "C" int qasr_check_expf_nonpos(int device, uint64_t *mismatches) {
    if (!mismatches) return fail(QASR_ERR_ARG, "bad arguments");
    int nd = 0, cur = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return fail(QASR_ERR_DEVICE, "no such HIP device");
    (void)hipGetDevice(&cur);
    if (hipSetDevice(device) != hipSuccess) return fail(QASR_ERR_DEVICE, "hipSetDevice failed");
    unsigned long long bad = ~0ull;
    const hipError_t e = check_expf_nonpos(&bad);
    (void)hipSetDevice(cur);
    if (e != hipSuccess) return fail(QASR_ERR_DEVICE, std::string("expf check: ") + hipGetErrorString(e));
    *mismatches = bad;
    return 0;
}

// -------------------------------------------------------------- loading
struct Up {
    std::string name;
    size_t bytes;
    void **dst;
    std::function<void(uint8_t *)> fill;
};

static bool check_shape(const gguf_tensor *t, std::vector<int64_t> ne, uint32_t want_type, std::string &err) {
    if (!t) { err = "missing tensor"; return false; }
    int64_t n = 1, m = 1;
    for (auto v : ne) n *= v;
    for (auto v : t->ne) m *= v;
    if (n != m) {
        err = "tensor " + t->name + ": expected " + std::to_string(n) + " elements, file has " + std::to_string(m);
        return false;
    }
    if (t->type != want_type) {
        err = "tensor " + t->name + ": unsupported ggml type " + std::to_string(t->type) +
              (want_type == DT_F32 ? " (expected F32)" : want_type == DT_Q8_0 ? " (expected Q8_0 like the other linear weights)"
                                                                              : " (expected F16)");
        return false;
    }
    return true;
}

extern "C" int qasr_model_load(const char *path, int device, qasr_model **out) {
    if (!path || !out) return fail(QASR_ERR_ARG, "null argument");
    *out = nullptr;
    const bool host_only = device == QASR_HOST_ONLY;
    if (!host_only) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(QASR_ERR_DEVICE, "no HIP device available");
        if (device < 0 || device >= ndev) return fail(QASR_ERR_ARG, "bad device index");
        HIPCHK(hipSetDevice(device));
    }
    GGUFFile f;
    if (!f.open(path)) return fail(QASR_ERR_IO, f.error());
    std::unique_ptr<qasr_model> m(new qasr_model());
    m->device = device;
    m->hp = read_hparams(f);
    const Hparams &hp = m->hp;
    std::string err;
    if (!m->tok.load(f, err)) return fail(QASR_ERR_FORMAT, err);
    if (hp.d_model / hp.enc_heads != 64 || hp.d_model % hp.enc_heads)
        return fail(QASR_ERR_FORMAT, "encoder head_dim must be 64");
    if (hp.head_dim != 128 || hp.n_head != 2 * hp.n_kv_head)
        return fail(QASR_ERR_FORMAT, "decoder must have head_dim 128 and GQA ratio 2");
    if (hp.n_mel != 128) return fail(QASR_ERR_FORMAT, "n_mel must be 128");
    if (hp.conv_ch % 32 || hp.dec_ffn % 16) return fail(QASR_ERR_FORMAT, "unsupported conv/ffn width");

    const int C = hp.conv_ch, D = hp.d_model, FF = hp.enc_ffn, H = hp.hidden, V = hp.vocab;
    const int QD = hp.n_head * 128, KD = hp.n_kv_head * 128, F = hp.dec_ffn;
    m->enc.resize(hp.enc_layers);
    m->dec.resize(hp.dec_layers);
    std::vector<Up> ups;
    auto T = [&](const std::string &n) { return f.tensor(n); };
    auto need = [&](const std::string &n, std::vector<int64_t> ne, uint32_t ty) -> const gguf_tensor * {
        const gguf_tensor *t = T(n);
        std::string e;
        if (!t) { if (err.empty()) err = "missing tensor: " + n; return nullptr; }
        if (!check_shape(t, ne, ty, e)) { if (err.empty()) err = e; return nullptr; }
        return t;
    };
    auto copy_f32 = [&](const std::string &n, int64_t len, float **dst) {
        const gguf_tensor *t = need(n, {len}, DT_F32);
        if (!t) return;
        ups.push_back({n, (size_t)len * 4, (void **)dst, [t, len](uint8_t *o) { memcpy(o, t->data, (size_t)len * 4); }});
    };
    auto copy_f16 = [&](const std::string &n, std::vector<int64_t> ne, uint16_t **dst) {
        const gguf_tensor *t = need(n, ne, DT_F16);
        if (!t) return;
        size_t bytes = t->nbytes;
        ups.push_back({n, bytes, (void **)dst, [t, bytes](uint8_t *o) { memcpy(o, t->data, bytes); }});
    };
    // conv kernels: [oc][ic][kh][kw] -> [oc][kh][kw][ic] (im2col K order of the implicit GEMM),
    // rows zero-padded to conv_kpad(IC) (the 8-phase tile's K % 128; gemm8p.h)
    auto conv_w = [&](const std::string &n, int IC, uint16_t **dst) {
        const gguf_tensor *t = need(n, {3, 3, IC, C}, DT_F16);
        if (!t) return;
        const int KP = conv_kpad(IC);
        ups.push_back({n, (size_t)C * KP * 2, (void **)dst, [t, IC, C, KP](uint8_t *o) {
                           const uint16_t *s = (const uint16_t *)t->data;
                           uint16_t *d = (uint16_t *)o;
                           memset(d, 0, (size_t)C * KP * 2);
                           for (int oc = 0; oc < C; oc++)
                               for (int ic = 0; ic < IC; ic++)
                                   for (int k = 0; k < 9; k++) d[(size_t)oc * KP + (size_t)k * IC + ic] = s[((size_t)oc * IC + ic) * 9 + k];
                       }});
    };
    copy_f16("audio.encoder.conv1.weight", {3, 3, 1, C}, &m->conv1_w);
    copy_f32("audio.encoder.conv1.bias", C, &m->conv1_b);
    conv_w("audio.encoder.conv2.weight", C, &m->conv2_w);
    copy_f32("audio.encoder.conv2.bias", C, &m->conv2_b);
    conv_w("audio.encoder.conv3.weight", C, &m->conv3_w);
    copy_f32("audio.encoder.conv3.bias", C, &m->conv3_b);
    // linear weights: every non-conv matrix except token_embd shares one type
    const gguf_tensor *probe = T("blk.0.attn_q.weight");
    const uint32_t LT = probe && probe->type == DT_Q8_0 ? DT_Q8_0 : DT_F16;
    m->q8 = LT == DT_Q8_0;
    // a linear weight [N][K] stacked from source tensors; rmap(r) -> {tensor, source row}
    auto lin = [&](const std::string &key, std::vector<const gguf_tensor *> src, int K, int N,
                   std::function<std::pair<int, int>(int)> rmap, uint16_t **dst, uint16_t **dst_d) {
        for (auto *t : src) if (!t) return;
        if (LT == DT_F16) {
            ups.push_back({key, (size_t)N * K * 2, (void **)dst, [src, K, N, rmap](uint8_t *o) {
                               for (int r = 0; r < N; r++) {
                                   const auto sr = rmap(r);
                                   memcpy(o + (size_t)r * K * 2, (const uint8_t *)src[sr.first]->data + (size_t)sr.second * K * 2,
                                          (size_t)K * 2);
                               }
                           }});
        } else {
            if (K % 32) { if (err.empty()) err = key + ": Q8_0 row length must be a multiple of 32"; return; }
            const int nb = K / 32;
            auto blocks = [src, nb, rmap](int r) {
                const auto sr = rmap(r);
                return (const uint8_t *)src[sr.first]->data + (size_t)sr.second * nb * 34;
            };
            ups.push_back({key, (size_t)N * K, (void **)dst, [blocks, K, N, nb](uint8_t *o) {
                               for (int r = 0; r < N; r++) {
                                   const uint8_t *b = blocks(r);
                                   for (int j = 0; j < nb; j++) memcpy(o + (size_t)r * K + 32 * j, b + 34 * j + 2, 32);
                               }
                           }});
            ups.push_back({key + ".d", (size_t)N * nb * 2, (void **)dst_d, [blocks, N, nb](uint8_t *o) {
                               for (int r = 0; r < N; r++) {
                                   const uint8_t *b = blocks(r);
                                   for (int j = 0; j < nb; j++) memcpy(o + ((size_t)r * nb + j) * 2, b + 34 * j, 2);
                               }
                           }});
        }
    };
    auto ident = [](int r) { return std::make_pair(0, r); };
    auto one = [&](const std::string &n, int K, int N, uint16_t **dst, uint16_t **dst_d) {
        lin(n, {need(n, {K, N}, LT)}, K, N, ident, dst, dst_d);
    };
    {   // conv_out: input feature c*16+h (src/audio_encoder.cpp:133-142).  F16: permuted
        // to h*C + c at load so the GEMM's A is conv3's [h][c] rows; Q8_0 keeps the
        // file order (blocks run along it) and the activation quantiser gathers.
        const gguf_tensor *t = need("audio.encoder.conv_out.weight", {(int64_t)C * 16, D}, LT);
        if (t && LT == DT_F16)
            ups.push_back({t->name, (size_t)D * C * 16 * 2, (void **)&m->conv_out_w, [t, C, D](uint8_t *o) {
                               const uint16_t *s = (const uint16_t *)t->data;
                               uint16_t *d = (uint16_t *)o;
                               for (int n = 0; n < D; n++)
                                   for (int c = 0; c < C; c++)
                                       for (int h = 0; h < 16; h++) d[(size_t)n * C * 16 + h * C + c] = s[(size_t)n * C * 16 + c * 16 + h];
                           }});
        else if (t)
            lin(t->name, {t}, 16 * C, D, ident, &m->conv_out_w, &m->conv_out_d);
    }
    for (int l = 0; l < hp.enc_layers; l++) {
        const std::string p = "audio.encoder.blk." + std::to_string(l) + ".";
        EncLayer &L = m->enc[l];
        const gguf_tensor *q = need(p + "attn_q.weight", {D, D}, LT), *k = need(p + "attn_k.weight", {D, D}, LT),
                          *v = need(p + "attn_v.weight", {D, D}, LT);
        const gguf_tensor *qb = need(p + "attn_q.bias", {D}, DT_F32), *kb = need(p + "attn_k.bias", {D}, DT_F32),
                          *vb = need(p + "attn_v.bias", {D}, DT_F32);
        lin(p + "qkv", {q, k, v}, D, 3 * D, [D](int r) { return std::make_pair(r / D, r % D); }, &L.wqkv, &L.wqkv_d);
        if (qb && kb && vb) {
            const size_t bb = (size_t)D * 4;
            ups.push_back({p + "bqkv", 3 * bb, (void **)&L.bqkv, [qb, kb, vb, bb](uint8_t *o) {
                               memcpy(o, qb->data, bb); memcpy(o + bb, kb->data, bb); memcpy(o + 2 * bb, vb->data, bb); }});
        }
        one(p + "attn_out.weight", D, D, &L.wo, &L.wo_d);
        copy_f32(p + "attn_out.bias", D, &L.bo);
        copy_f32(p + "attn_norm.weight", D, &L.ln1_w);
        copy_f32(p + "attn_norm.bias", D, &L.ln1_b);
        one(p + "ffn_up.weight", D, FF, &L.w1, &L.w1_d);
        copy_f32(p + "ffn_up.bias", FF, &L.b1);
        one(p + "ffn_down.weight", FF, D, &L.w2, &L.w2_d);
        copy_f32(p + "ffn_down.bias", D, &L.b2);
        copy_f32(p + "ffn_norm.weight", D, &L.ln2_w);
        copy_f32(p + "ffn_norm.bias", D, &L.ln2_b);
    }
    copy_f32("audio.encoder.ln_post.weight", D, &m->ln_post_w);
    copy_f32("audio.encoder.ln_post.bias", D, &m->ln_post_b);
    one("audio.encoder.proj1.weight", D, D, &m->proj1_w, &m->proj1_d);
    copy_f32("audio.encoder.proj1.bias", D, &m->proj1_b);
    one("audio.encoder.proj2.weight", D, H, &m->proj2_w, &m->proj2_d);
    copy_f32("audio.encoder.proj2.bias", H, &m->proj2_b);
    copy_f16("token_embd.weight", {H, V}, &m->embd);   // tied LM head (src/text_decoder.cpp:264-265), F16 in both file types
    if (hp.aligner) {   // classify head: output.weight as [hidden][classify_num] (src/forced_aligner.cpp:274-277, 1073)
        const gguf_tensor *t = T("output.weight");
        const int NC = hp.classify_num;
        if (!t || t->type != DT_F16 || t->ne.size() != 2 || t->ne[0] != H || t->ne[1] < NC || NC <= 0) {
            if (err.empty()) err = "aligner: output.weight must be F16 [hidden][>= classify_num]";
        } else {
            m->cls_rows = (NC + 63) / 64 * 64;   // the GEMM tiles 64 columns; padded rows never win the argmax
            const size_t bytes = (size_t)m->cls_rows * H * 2;
            ups.push_back({"output.weight", bytes, (void **)&m->cls_w, [t, NC, H, bytes](uint8_t *o) {
                               memset(o, 0, bytes);
                               memcpy(o, t->data, (size_t)NC * H * 2);
                           }});
        }
    }
    copy_f32("output_norm.weight", H, &m->out_norm);
    for (int l = 0; l < hp.dec_layers; l++) {
        const std::string p = "blk." + std::to_string(l) + ".";
        DecLayer &L = m->dec[l];
        copy_f32(p + "attn_norm.weight", H, &L.attn_norm);
        copy_f32(p + "attn_q_norm.weight", 128, &L.q_norm);
        copy_f32(p + "attn_k_norm.weight", 128, &L.k_norm);
        copy_f32(p + "ffn_norm.weight", H, &L.ffn_norm);
        const gguf_tensor *q = need(p + "attn_q.weight", {H, QD}, LT), *k = need(p + "attn_k.weight", {H, KD}, LT),
                          *v = need(p + "attn_v.weight", {H, KD}, LT);
        lin(p + "qkv", {q, k, v}, H, QD + 2 * KD,
            [QD, KD](int r) { return r < QD ? std::make_pair(0, r) : r < QD + KD ? std::make_pair(1, r - QD) : std::make_pair(2, r - QD - KD); },
            &L.wqkv, &L.wqkv_d);
        one(p + "attn_output.weight", QD, H, &L.wo, &L.wo_d);
        const gguf_tensor *gt = need(p + "ffn_gate.weight", {H, F}, LT), *ut = need(p + "ffn_up.weight", {H, F}, LT);
        // interleave 16-row blocks: [gate 16q..16q+15 | up 16q..16q+15] -> SwiGLU in one epilogue
        lin(p + "gu", {gt, ut}, H, 2 * F, [](int r) { return std::make_pair((r % 32) < 16 ? 0 : 1, 16 * (r / 32) + (r % 16)); },
            &L.wgu, &L.wgu_d);
        one(p + "ffn_down.weight", F, H, &L.wd, &L.wd_d);
    }
    if (!err.empty()) return fail(QASR_ERR_FORMAT, err);
    // constant tables
    std::vector<uint16_t> lut;
    gelu_table(lut);
    ups.push_back({"gelu", lut.size() * 2, (void **)&m->gelu, [lut](uint8_t *o) { memcpy(o, lut.data(), lut.size() * 2); }});
    std::vector<float> pe;
    sinusoidal_pe(pe, 13, D);   // a 100-frame chunk yields at most 13 frames
    ups.push_back({"pe", pe.size() * 4, (void **)&m->pe, [pe](uint8_t *o) { memcpy(o, pe.data(), pe.size() * 4); }});
    std::vector<float> fl;
    mel_filters(fl);
    ups.push_back({"filters", fl.size() * 4, (void **)&m->filters, [fl](uint8_t *o) { memcpy(o, fl.data(), fl.size() * 4); }});
    std::vector<double> tw, hn;
    dft_twiddles(tw);
    hann_window(hn);
    ups.push_back({"tw", tw.size() * 8, (void **)&m->tw, [tw](uint8_t *o) { memcpy(o, tw.data(), tw.size() * 8); }});
    ups.push_back({"hann", hn.size() * 8, (void **)&m->hann, [hn](uint8_t *o) { memcpy(o, hn.data(), hn.size() * 8); }});

    if (host_only) {   // hparams + tokenizer only: text helpers, validation, tests without a GPU
        *out = m.release();
        return 0;
    }
    size_t total = 0;
    std::vector<size_t> offs(ups.size());
    for (size_t i = 0; i < ups.size(); i++) {
        offs[i] = total;
        total += (ups[i].bytes + 255) / 256 * 256;
    }
    HIPCHK(hipMalloc((void **)&m->arena, total));
    m->arena_bytes = total;
    std::vector<uint8_t> host;
    for (size_t i = 0; i < ups.size(); i++) {
        host.resize(ups[i].bytes);
        ups[i].fill(host.data());
        HIPCHK(hipMemcpy(m->arena + offs[i], host.data(), ups[i].bytes, hipMemcpyHostToDevice));
        *ups[i].dst = m->arena + offs[i];
    }
    *out = m.release();
    return 0;
}

extern "C" void qasr_model_free(qasr_model *m) { delete m; }

extern "C" int qasr_model_hparams(const qasr_model *m, qasr_hparams *o) {
    if (!m || !o) return fail(QASR_ERR_ARG, "null argument");
    const Hparams &h = m->hp;
    *o = qasr_hparams{h.enc_layers, h.d_model, h.enc_heads, h.enc_ffn, h.conv_ch, h.n_mel, h.enc_eps,
                      h.vocab, h.hidden, h.dec_layers, h.n_head, h.n_kv_head, h.head_dim, h.dec_ffn, h.rms_eps, h.rope_theta,
                      h.eos_id, h.pad_id, h.audio_start_id, h.audio_end_id, h.audio_pad_id, h.weight_type,
                      h.aligner ? h.classify_num : 0, h.timestamp_id};
    return 0;
}

extern "C" int64_t qasr_model_device_bytes(const qasr_model *m) { return m ? (int64_t)m->arena_bytes : 0; }

// --------------------------------------------------------------- context
extern "C" int qasr_ctx_create(qasr_model *m, int max_batch, int max_ctx, qasr_ctx **out) {
    if (!m || !out || max_batch <= 0 || max_ctx <= 0) return fail(QASR_ERR_ARG, "bad context arguments");
    if (!m->arena) return fail(QASR_ERR_STATE, "model was loaded host-only (device QASR_HOST_ONLY)");
    *out = nullptr;
    HIPCHK(hipSetDevice(m->device));
    std::unique_ptr<qasr_ctx> c(new qasr_ctx());
    c->m = m;
    c->max_batch = max_batch;
    c->max_ctx = max_ctx;
    HIPCHK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    for (auto &e : c->ev) HIPCHK(hipEventCreate(&e));
    const Hparams &hp = m->hp;
    // + padding rows: fa_exact.hip's chains read V a few batches past the context
    const size_t kv = (size_t)hp.dec_layers * max_batch * hp.n_kv_head * max_ctx * 128 + kKvPadRows * 128;
    int rc = 0;
    if ((rc = dev_alloc(c.get(), (void **)&c->kc, kv * 2)) || (rc = dev_alloc(c.get(), (void **)&c->vc, kv * 2))) return rc;
    const size_t vt = (size_t)hp.dec_layers * layer_vt(c.get());
    if ((rc = dev_alloc(c.get(), (void **)&c->vt, vt * 2))) return rc;
    HIPCHK(hipMemset(c->vt, 0, vt * 2));
    std::vector<float> rope;
    rope_table(rope, max_ctx, 128, hp.rope_theta);
    if ((rc = dev_alloc(c.get(), (void **)&c->rope, rope.size() * 4))) return rc;
    HIPCHK(hipMemcpy(c->rope, rope.data(), rope.size() * 4, hipMemcpyHostToDevice));
    const int B = max_batch, QD = hp.n_head * 128, KD = hp.n_kv_head * 128;
    c->max_splits = (max_ctx + decode_split_len() - 1) / decode_split_len();
    if (c->max_splits > decode_max_splits())
        return fail(QASR_ERR_ARG, "max_ctx exceeds " + std::to_string(decode_max_splits() * decode_split_len()));
    const char *ng = getenv("QASR_NO_GRAPH");
    c->eager = ng && ng[0] == '1';
#ifdef QASR_DIAG_SKIP   // diagnostic builds only (tools/): drops decode kernels to price them -- wrong tokens
    if (const char *ds = getenv("QASR_DEV_SKIP")) c->dev_skip = atoi(ds);
#endif
    // fused-launch options: environment defaults, per-context overrides via qasr_ctx_set_option
    for (const auto &o : fuse_options()) {
        if (const char *e = getenv(o.env)) c->fuse.*(o.field) = atoi(e);
    }
    fused_slots(c->fuse);   // co-residency on this context's device
    if (const char *tp = getenv("QASR_DEV_TRACE")) {
        c->trace_path = tp;
        if (const char *tl = getenv("QASR_DEV_TRACE_LAYER")) c->trace_layer = atoi(tl);
        if ((rc = dev_alloc(c.get(), (void **)&c->d_trace, 6 * 4096 * 8 * 8))) return rc;
        HIPCHK(hipMemset(c->d_trace, 0, 6 * 4096 * 8 * 8));
    }
    c->hist_cap = max_ctx;
    if ((rc = dev_alloc(c.get(), (void **)&c->d_tok, B * 4)) || (rc = dev_alloc(c.get(), (void **)&c->d_hist, (size_t)B * max_ctx * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_pos, B * 4)) || (rc = dev_alloc(c.get(), (void **)&c->d_nkv, B * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_slot, B * 4)) || (rc = dev_alloc(c.get(), (void **)&c->d_step, 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_x, (size_t)B * hp.hidden * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_xh, (size_t)B * hp.hidden * 2)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_qkv, (size_t)B * (QD + 2 * KD) * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_q, (size_t)B * QD * 2)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_att, (size_t)B * QD * 2)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_act, (size_t)B * hp.dec_ffn * 2)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_att32, (size_t)B * QD * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_act32, (size_t)B * hp.dec_ffn * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_q8a, (size_t)B * std::max(QD, std::max(hp.hidden, hp.dec_ffn)))) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_q8d, (size_t)B * std::max(QD, std::max(hp.hidden, hp.dec_ffn)) / 32 * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_x32, (size_t)B * std::max(QD, std::max(hp.hidden, hp.dec_ffn)) * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_q8n, (size_t)B * hp.hidden)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_q8nd, (size_t)B * hp.hidden / 32 * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_part, (size_t)B * hp.n_kv_head * c->max_splits * 2 * 132 * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_counter, (size_t)B * hp.n_kv_head * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_scores, (size_t)B * hp.n_head * max_ctx * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_qcnt, (size_t)hp.n_kv_head * 8 * 16 * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_attdone, (size_t)hp.dec_layers * 128 * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_gran, (size_t)(QD + 2 * KD) * 8)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_sgran, (size_t)hp.n_head * sgran_ld(max_ctx) * 8)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_ffncnt, (size_t)hp.dec_layers * 1024 * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_done, 4)) || (rc = dev_alloc(c.get(), (void **)&c->d_err, 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_pstamp, (size_t)max_ctx * kStampRec * 8)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_logits, (size_t)B * hp.vocab * 4)) ||
        (rc = dev_alloc(c.get(), (void **)&c->d_amax, (size_t)B * 8)))
        return rc;
    std::vector<int> slots(B);
    for (int b = 0; b < B; b++) slots[b] = b;
    HIPCHK(hipMemcpy(c->d_slot, slots.data(), B * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(c->d_counter, 0, (size_t)B * hp.n_kv_head * 4));
    HIPCHK(hipMemset(c->d_qcnt, 0, (size_t)hp.n_kv_head * 8 * 16 * 4));
    HIPCHK(hipMemset(c->d_attdone, 0, (size_t)hp.dec_layers * 128 * 4));
    HIPCHK(hipMemset(c->d_gran, 0, (size_t)(QD + 2 * KD) * 8));
    HIPCHK(hipMemset(c->d_sgran, 0, (size_t)hp.n_head * sgran_ld(max_ctx) * 8));
    HIPCHK(hipMemset(c->d_ffncnt, 0, (size_t)hp.dec_layers * 1024 * 4));
    HIPCHK(hipMemset(c->d_done, 0, 4));
    HIPCHK(hipMemset(c->d_err, 0, 4));
    c->fuse.err = c->d_err;
    HIPCHK(hipMemset(c->kc, 0, kv * 2));   // decode attention reads whole splits and masks: keep every row finite
    HIPCHK(hipMemset(c->vc, 0, kv * 2));
    HIPCHK(hipMemset(c->d_amax, 0, (size_t)B * 8));
    *out = c.release();
    return 0;
}

extern "C" void qasr_ctx_free(qasr_ctx *c) { delete c; }

extern "C" int qasr_ctx_set_option(qasr_ctx *c, const char *name, int value) {
    if (!c || !name) return fail(QASR_ERR_ARG, "bad arguments");
    const std::string n = name;
    if (n == "probe_layer") {
        if (value < 0 || value >= c->m->hp.dec_layers) return fail(QASR_ERR_ARG, "probe_layer out of range");
        c->probe_layer = value;
        c->drop_graphs();
        c->graph_probe_group = -1;
        return 0;
    }
    if (n == "probe_stride") {
        if (value < 1) return fail(QASR_ERR_ARG, "probe_stride must be >= 1");
        c->probe_stride = value;
        return 0;
    }
    if (n == "dec_layers") {
        if (value < 0 || value > c->m->hp.dec_layers) return fail(QASR_ERR_ARG, "dec_layers out of range");
        c->dbg_layers = value;
        c->drop_graphs();
        return 0;
    }
    for (const auto &o : fuse_options())
        if (n == o.name) {
            if (n == "poll_limit" && value <= 0) return fail(QASR_ERR_ARG, "poll_limit must be positive");
            c->fuse.*(o.field) = value;
            c->drop_graphs();   // captured steps hold the old launch configuration
            HIPCHK(hipSetDevice(c->m->device));   // arrival counters back to rest
            const int rc = reset_counters(c);
            if (rc) return rc;
            HIPCHK(hipStreamSynchronize(c->st));
            return 0;
        }
    return fail(QASR_ERR_ARG, "unknown option '" + n + "'");
}

extern "C" int qasr_ctx_get_option(const qasr_ctx *c, const char *name, int *value) {
    if (!c || !name || !value) return fail(QASR_ERR_ARG, "bad arguments");
    const std::string n = name;
    if (n == "dec_layers") { *value = c->dbg_layers; return 0; }
    if (n == "probe_layer") { *value = c->probe_layer; return 0; }
    if (n == "probe_stride") { *value = c->probe_stride; return 0; }
    if (n == "slots_ffn") { *value = c->fuse.slots_ffn; return 0; }
    if (n == "fused_mode") { *value = c->last_fmode; return 0; }
    if (n == "fused_exact") { *value = c->last_fx; return 0; }
    if (n == "attn_path") { *value = c->last_attn; return 0; }
    if (n == "slots_qkv") { *value = std::min(c->fuse.slots_qkv64, c->fuse.slots_qkv128); return 0; }
    for (const auto &o : fuse_options())
        if (n == o.name) { *value = c->fuse.*(o.field); return 0; }
    return fail(QASR_ERR_ARG, "unknown option '" + n + "'");
}

extern "C" int qasr_debug_read(qasr_ctx *c, const char *buffer, void *dst, int64_t bytes) {
    if (!c || !buffer || !dst || bytes < 0) return fail(QASR_ERR_ARG, "bad arguments");
    const Hparams &hp = c->m->hp;
    const int64_t B = c->max_batch, QD = hp.n_head * 128, KD = hp.n_kv_head * 128;
    const std::string n = buffer;
    const void *src = nullptr;
    int64_t cap = 0;
    if (n == "x") { src = c->d_x; cap = B * hp.hidden * 4; }
    else if (n == "act") { src = c->d_act; cap = B * hp.dec_ffn * 2; }
    else if (n == "qkv") { src = c->d_qkv; cap = B * (QD + 2 * KD) * 4; }
    else if (n == "att") { src = c->d_att; cap = B * QD * 2; }
    else return fail(QASR_ERR_ARG, "unknown buffer '" + n + "'");
    if (bytes > cap) return fail(QASR_ERR_ARG, "read past the buffer");
    HIPCHK(hipSetDevice(c->m->device));
    if (n == "qkv" && c->qkv_in_gran) {   // the last layer's QKV went out as {value, tag} granules (batch 1)
        std::vector<unsigned long long> g(QD + 2 * KD);
        HIPCHK(hipMemcpyAsync(g.data(), c->d_gran, g.size() * 8, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        std::vector<uint32_t> v(B * (QD + 2 * KD), 0u);
        for (size_t i = 0; i < g.size(); i++) v[i] = (uint32_t)g[i];
        memcpy(dst, v.data(), bytes);
        return 0;
    }
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// ------------------------------------------------------------ size helpers
extern "C" int qasr_mel_frames(int n) { return mel_frames(n); }
extern "C" int qasr_encoder_frames(int T) { return encoder_frames(T); }
extern "C" int qasr_prompt_len(int n) { return n + 15; }
extern "C" int qasr_align_prompt_len(int n_samples, int n_text) {
    return n_text + 2 + feat_extract_output_lengths(mel_frames(n_samples));
}
extern "C" int qasr_build_prompt(const qasr_model *m, int n_audio, int32_t *ids, int *audio_pos) {
    Hparams hp = m ? m->hp : Hparams();
    std::vector<int32_t> p = build_prompt(hp, n_audio, {}, audio_pos);
    if (ids) memcpy(ids, p.data(), p.size() * 4);
    return (int)p.size();
}

// =================================================================== stages
// mel for B clips whose PCM is already in c->pcm (offsets/lengths given);
// result in c->mel as B blocks [128][T_b].
static int run_mel(qasr_ctx *c, const std::vector<long> &off, const std::vector<int> &n, std::vector<long> &mel_off,
                   std::vector<int> &T, const float *d_pcm = nullptr) {
    qasr_model *m = c->m;
    const int B = (int)n.size();
    std::vector<MelClip> clips(B);
    std::vector<int2> blocks;
    long tmp_total = 0, out_total = 0;
    T.resize(B);
    mel_off.resize(B);
    const int fpb = mel_frames_per_block();
    for (int b = 0; b < B; b++) {
        const int TF = n[b] / 160 + 1;
        clips[b] = MelClip{off[b], n[b], TF, tmp_total, out_total};
        T[b] = TF - 1;
        mel_off[b] = out_total;
        tmp_total += 128L * TF;
        out_total += 128L * (TF - 1);
        for (int f = 0; f < TF; f += fpb) blocks.push_back(make_int2(b, f));
    }
    int rc;
    if ((rc = upload(c, c->melclips, clips)) || (rc = upload(c, c->melblocks, blocks)) ||
        (rc = ensure(c, c->meltmp, tmp_total * 8)) || (rc = ensure(c, c->mel, std::max<long>(out_total, 1) * 4)) ||
        (rc = ensure(c, c->melmax, B * 8)))
        return rc;
    HIPCHK(hipMemsetAsync(c->melmax.p, 0, B * 8, c->st));
    launch_mel(d_pcm ? d_pcm : c->pcm.as<float>(), c->melclips.as<MelClip>(), B, blocks.empty() ? nullptr : c->melblocks.as<int2>(),
               (int)blocks.size(), m->tw, m->hann, m->filters, c->meltmp.as<double>(), c->melmax.as<unsigned long long>(),
               c->mel.as<float>(), c->st);
    HIPCHK(hipGetLastError());
    return 0;
}

// encoder over B clips whose mel sits at d_mel + mel_off[b] ([128][T_b]).
// conv_only: stop after conv_out + PE (output [sum N][d_model] in c->ex).
// no_chunk: AudioEncoder::encode_no_chunk (src/audio_encoder.cpp:603-852): the
// conv stack over each clip's frames as one chunk, PE positions 0 .. N-1 (ASR)
static int run_encoder(qasr_ctx *c, const float *d_mel, const std::vector<long> &mel_off, const std::vector<int> &T,
                       bool conv_only, std::vector<int> &Nb, bool no_chunk = false) {
    qasr_model *m = c->m;
    const Hparams &hp = m->hp;
    const int B = (int)T.size(), C = hp.conv_ch, D = hp.d_model, FF = hp.enc_ffn;
    std::vector<ChunkDesc> ch;
    std::vector<int> s1, s2, s3, pepos;
    int r1 = 0, r2 = 0, r3 = 0, er = 0;
    Nb.assign(B, 0);
    // ASR: each chunk on its own length (src/audio_encoder.cpp:331-409).  Aligner:
    // every chunk zero-padded to 100 frames, the valid frames of the (short)
    // last one kept (src/forced_aligner.cpp:601-735).  One clip: the valid
    // conv_out rows are the leading rows.  Several clips: a clip's short last
    // chunk leaves padded rows before the next clip's, so conv_out runs over
    // every padded row (PE position = row within its chunk, as for the valid
    // ones) and the valid rows are gathered after it.
    const bool al = hp.aligner;
    if (no_chunk && al) return fail(QASR_ERR_ARG, "encode_no_chunk: ASR models only");
    const bool al_gather = al && B > 1;
    std::vector<int> pepos_pad, gidx;
    for (int b = 0; b < B; b++) {
        const int CH = no_chunk ? std::max(T[b], 1) : 100;
        for (int s = 0; s < T[b]; s += CH) {
            ChunkDesc d;
            d.mel_off = mel_off[b] + s;
            d.T = T[b];
            d.Lv = std::min(CH, T[b] - s);
            d.L = al ? 100 : d.Lv;
            d.W1 = (d.L - 1) / 2 + 1;
            d.W2 = (d.W1 - 1) / 2 + 1;
            d.W3 = (d.W2 - 1) / 2 + 1;
            d.row1 = r1; d.row2 = r2; d.row3 = r3; d.enc_row = er;
            s1.push_back(r1); s2.push_back(r2); s3.push_back(r3);
            const int valid = chunk_out_len(d.Lv);
            if (al_gather) {
                for (int w = 0; w < d.W3; w++) pepos_pad.push_back(w);
                for (int w = 0; w < valid; w++) gidx.push_back(r3 / 16 + w);
            }
            r1 += 64 * d.W1; r2 += 32 * d.W2; r3 += 16 * d.W3; er += valid;
            for (int w = 0; w < valid; w++) pepos.push_back(w);
            Nb[b] += valid;
            ch.push_back(d);
        }
    }
    const int NC = (int)ch.size(), N = er;
    if (N == 0) return 0;
    int rc;
    const float *pe_tab = m->pe;   // 13 positions: a 100-frame chunk's
    if (no_chunk) {
        int npos = 0;
        for (int v : Nb) npos = std::max(npos, v);
        if (npos > c->pebig_rows) {
            std::vector<float> pe;
            sinusoidal_pe(pe, npos, D);
            if ((rc = ensure(c, c->pebig, pe.size() * 4))) return rc;
            HIPCHK(hipMemcpy(c->pebig.p, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
            c->pebig_rows = npos;
        }
        pe_tab = c->pebig.as<float>();
    }
    const int NP = r3 / 16;   // conv_out rows over every (padded) chunk row
    if (al_gather && ((rc = upload(c, c->gidx, gidx)) || (rc = ensure(c, c->exp_, (size_t)NP * D * 4)))) return rc;
    if ((rc = upload(c, c->chunks, ch)) || (rc = upload(c, c->rs1, s1)) || (rc = upload(c, c->rs2, s2)) ||
        (rc = upload(c, c->rs3, s3)) || (rc = upload(c, c->pepos, al_gather ? pepos_pad : pepos)) ||
        (rc = ensure(c, c->act1, (size_t)r1 * C * 2)) || (rc = ensure(c, c->act2, (size_t)r2 * C * 2)) ||
        (rc = ensure(c, c->act3, (size_t)r3 * C * 2)) || (rc = ensure(c, c->ex, (size_t)N * D * 4)) ||
        (rc = ensure(c, c->exh, (size_t)N * std::max(D, FF) * 2)) || (rc = ensure(c, c->eqkv, (size_t)N * 3 * D * 4)) ||
        (rc = ensure(c, c->eatt, (size_t)N * D * 2)) || (rc = ensure(c, c->eff, (size_t)N * FF * 2)) ||
        (rc = ensure(c, c->feats, (size_t)N * hp.hidden * 4)))
        return rc;
    hipStream_t s = c->st;
    int max_w1 = 0;
    for (const ChunkDesc &d : ch) max_w1 = std::max(max_w1, d.W1);
    launch_conv1(d_mel, c->chunks.as<ChunkDesc>(), c->rs1.as<int>(), NC, r1, m->conv1_w, m->conv1_b, m->gelu, C,
                 c->act1.as<uint16_t>(), s, max_w1);
    GemmArgs g{};
    g.chunks = c->chunks.as<ChunkDesc>();
    g.n_chunks = NC;
    g.C = C;
    g.gelu = m->gelu;
    // conv2: act1 (NHWC, H=64) -> act2 (NHWC, H=32)
    g.A = c->act1.as<uint16_t>(); g.W = m->conv2_w; g.ldw = conv_kpad(C); g.M = r2; g.N = C; g.K = 9 * C;
    g.row_start = c->rs2.as<int>(); g.bias = m->conv2_b; g.out_f16 = c->act2.as<uint16_t>(); g.ldo16 = C;
    launch_gemm_c(c, AM_CONV2, EPI_GELU_F16, g, s);
    // conv3: act2 -> act3 rows ordered (chunk, w, h) so conv_out's A is dense
    g.A = c->act2.as<uint16_t>(); g.W = m->conv3_w; g.M = r3; g.row_start = c->rs3.as<int>(); g.bias = m->conv3_b;
    g.out_f16 = c->act3.as<uint16_t>();
    launch_gemm_c(c, AM_CONV3, EPI_GELU_F16, g, s);
    const bool q8 = m->q8;
    const int MO = al_gather ? NP : N;
    if (q8 && (rc = ensure_q8(c, MO, std::max(16 * C, std::max(D, FF)), D))) return rc;
    // conv_out (no bias) + per-chunk sinusoidal PE (src/audio_encoder.cpp:147-149, :400-404)
    GemmArgs o{};
    o.M = MO; o.N = D; o.K = 16 * C;
    o.out_f32 = al_gather ? c->exp_.as<float>() : c->ex.as<float>(); o.ldo = D; o.pe = pe_tab; o.pe_pos = c->pepos.as<int>();
    if (q8) {
        gemm_q8(c, EPI_F32, o, nullptr, c->act3.as<uint16_t>(), 16 * C, C, m->conv_out_w, m->conv_out_d, s);
    } else {
        o.A = c->act3.as<uint16_t>(); o.lda = 16 * C; o.W = m->conv_out_w; o.ldw = 16 * C;
        launch_gemm_c(c, AM_DENSE, EPI_F32, o, s);
    }
    if (al_gather) launch_gather_rows(c->exp_.as<float>(), c->gidx.as<int>(), N, D, c->ex.as<float>(), s);
    HIPCHK(hipGetLastError());
    if (c->profile_on) HIPCHK(hipEventRecord(c->ev[5], s));   // conv front-end | transformer
    if (conv_only) return 0;

    // attention segments: whole clips (ASR: full attention, src/audio_encoder.cpp:466-486)
    // or the aligner's block-diagonal windows of 13 * (800 / 100) = 104 frames
    // (src/forced_aligner.cpp:737-766)
    std::vector<int> sst, sln;
    int acc = 0, maxn = 0;
    for (int b = 0; b < B; b++) {
        const int win = al ? 104 : std::max(Nb[b], 1);
        for (int o = 0; o < Nb[b]; o += win) {
            sst.push_back(acc + o);
            sln.push_back(std::min(win, Nb[b] - o));
            maxn = std::max(maxn, sln.back());
        }
        acc += Nb[b];
    }
    const int NS = (int)sst.size();
    std::vector<int> segs(sst);
    segs.insert(segs.end(), sln.begin(), sln.end());
    if ((rc = upload(c, c->segs, segs))) return rc;
    float *x = c->ex.as<float>();
    uint16_t *xh = c->exh.as<uint16_t>();
    float *x32 = q8 ? c->x32.as<float>() : nullptr;
    // y = act W^T with the model's weight type: F16 takes the fp16 activation
    // (a16), Q8_0 quantises the fp32 (a32) or fp16 one
    auto linear = [&](int epi, GemmArgs g, const float *a32, const uint16_t *a16, int lda, const uint16_t *W, const uint16_t *Wd) {
        if (q8) { gemm_q8(c, epi, g, a32, a32 ? nullptr : a16, lda, 0, W, Wd, s); return; }
        g.A = a16; g.lda = lda; g.W = W; g.ldw = g.K;
        launch_gemm_c(c, AM_DENSE, epi, g, s);
    };
    for (int l = 0; l < hp.enc_layers; l++) {
        const EncLayer &L = m->enc[l];
        launch_layernorm_f16(x, N, D, L.ln1_w, L.ln1_b, hp.enc_eps, xh, s, x32);
        GemmArgs q{};
        q.M = N; q.N = 3 * D; q.K = D; q.bias = L.bqkv; q.out_f32 = c->eqkv.as<float>(); q.ldo = 3 * D;
        linear(EPI_F32, q, x32, xh, D, L.wqkv, L.wqkv_d);
        launch_enc_attention(c->eqkv.as<float>(), c->segs.as<int>(), c->segs.as<int>() + NS, NS, maxn, D, hp.enc_heads,
                             c->eatt.as<uint16_t>(), s, x32, c->fuse.enc_attn_f32 != 0);
        GemmArgs op{};
        op.M = N; op.N = D; op.K = D; op.bias = L.bo; op.res = x; op.ldr = D; op.out_f32 = x; op.ldo = D;
        linear(EPI_F32, op, x32, c->eatt.as<uint16_t>(), D, L.wo, L.wo_d);
        launch_layernorm_f16(x, N, D, L.ln2_w, L.ln2_b, hp.enc_eps, xh, s, x32);
        GemmArgs f1{};
        f1.M = N; f1.N = FF; f1.K = D; f1.bias = L.b1; f1.gelu = m->gelu; f1.out_f16 = c->eff.as<uint16_t>(); f1.ldo16 = FF;
        linear(EPI_GELU_F16, f1, x32, xh, D, L.w1, L.w1_d);
        GemmArgs f2{};   // GELU output is fp16-exact (LUT): the Q8_0 path quantises it as is
        f2.M = N; f2.N = D; f2.K = FF; f2.bias = L.b2; f2.res = x; f2.ldr = D; f2.out_f32 = x; f2.ldo = D;
        linear(EPI_F32, f2, nullptr, c->eff.as<uint16_t>(), FF, L.w2, L.w2_d);
    }
    launch_layernorm_f16(x, N, D, m->ln_post_w, m->ln_post_b, hp.enc_eps, xh, s, x32);
    GemmArgs p1{};
    p1.M = N; p1.N = D; p1.K = D; p1.bias = m->proj1_b; p1.gelu = m->gelu; p1.out_f16 = c->eatt.as<uint16_t>(); p1.ldo16 = D;
    linear(EPI_GELU_F16, p1, x32, xh, D, m->proj1_w, m->proj1_d);
    GemmArgs p2{};
    p2.M = N; p2.N = hp.hidden; p2.K = D; p2.bias = m->proj2_b; p2.out_f32 = c->feats.as<float>(); p2.ldo = hp.hidden;
    linear(EPI_F32, p2, nullptr, c->eatt.as<uint16_t>(), D, m->proj2_w, m->proj2_d);
    HIPCHK(hipGetLastError());
    return declined_check("encoder");
}

// embedding gather + audio splice + decoder layer stack over the prompt rows of
// B sequences (positions 0..P_b-1, KV cache of sequence b reset); leaves the
// final hidden rows in c->px.  Row tables live in c->prow:
// [row_seq | row_pos | row_audio] (3*rows ints) + [seq_row0 | seq_len | seq_slot].
static int prefill_layers(qasr_ctx *c, const std::vector<int32_t> &ids, const std::vector<int> &P, const float *d_feats,
                          const std::vector<int> &audio_pos, const std::vector<int> &N, const std::vector<int> *slots,
                          const std::vector<int> *pos0 = nullptr) {
    qasr_model *m = c->m;
    const Hparams &hp = m->hp;
    const int B = (int)P.size(), H = hp.hidden, QD = hp.n_head * 128, KD = hp.n_kv_head * 128, F = hp.dec_ffn;
    if (B > c->max_batch) return fail(QASR_ERR_ARG, "batch exceeds context max_batch");
    if (slots)
        for (int v : *slots)
            if (v < 0 || v >= c->max_batch) return fail(QASR_ERR_ARG, "KV-cache slot out of range");
    int rows = 0, maxp = 0;
    auto p0 = [&](int b) { return pos0 ? (*pos0)[b] : 0; };   // a chunk after p0(b) cached tokens
    for (int b = 0; b < B; b++) {
        if (P[b] <= 0) return fail(QASR_ERR_ARG, "empty prompt");
        if (p0(b) < 0 || p0(b) + P[b] > c->max_ctx) return fail(QASR_ERR_ARG, "Context length exceeded");
        rows += P[b];
        maxp = std::max(maxp, P[b]);
    }
    if (pos0 && (m->hp.aligner || !c->fuse.fa_exact_prefill))   // (the chunk form is built on the exact kernel)
        for (int b = 0; b < B; b++)
            if (p0(b)) return fail(QASR_ERR_ARG, "a chunk after cached tokens needs the exact prefill attention (ASR model)");
    std::vector<int> tab(3 * rows + 4 * B), lastrow(B);
    int r = 0, fr = 0;
    for (int b = 0; b < B; b++) {
        const bool splice = d_feats && N[b] > 0 && audio_pos[b] >= 0 && audio_pos[b] + N[b] <= P[b];
        for (int t = 0; t < P[b]; t++, r++) {
            tab[r] = slots ? (*slots)[b] : b;   // the KV-cache slot the row writes
            tab[rows + r] = p0(b) + t;
            tab[2 * rows + r] = (splice && t >= audio_pos[b] && t < audio_pos[b] + N[b]) ? fr + (t - audio_pos[b]) : -1;
        }
        fr += N[b];
        lastrow[b] = r - 1;
    }
    int acc = 0;
    for (int b = 0; b < B; b++) {   // seq_row0 | seq_len | seq_slot | seq_pos0
        tab[3 * rows + b] = acc;
        tab[3 * rows + B + b] = P[b];
        tab[3 * rows + 2 * B + b] = slots ? (*slots)[b] : b;
        tab[3 * rows + 3 * B + b] = p0(b);
        acc += P[b];
    }
    int rc;
    if ((rc = upload(c, c->prow, tab)) || (rc = upload(c, c->plast, lastrow)) || (rc = upload(c, c->pids, ids)) ||
        (rc = ensure(c, c->px, (size_t)rows * H * 4)) || (rc = ensure(c, c->pxh, (size_t)rows * std::max(H, F) * 2)) ||
        (rc = ensure(c, c->pqkv, (size_t)rows * (QD + 2 * KD) * 4)) || (rc = ensure(c, c->pq, (size_t)rows * QD * 2)) ||
        (rc = ensure(c, c->patt, (size_t)rows * QD * 2)) || (rc = ensure(c, c->pact, (size_t)rows * F * 2)))
        return rc;
    const bool al = hp.aligner;   // fp32 Q / K scores (src/forced_aligner.cpp:1041-1046)
    if (al && ((rc = ensure(c, c->pq32, (size_t)rows * QD * 4)) || (rc = ensure(c, c->pk32, (size_t)rows * KD * 4)))) return rc;
    hipStream_t s = c->st;
    const int *d_seq = c->prow.as<int>(), *d_pos = d_seq + rows, *d_aud = d_seq + 2 * rows;
    const int *d_srow0 = d_seq + 3 * rows, *d_slen = d_srow0 + B, *d_sslot = d_slen + B, *d_spos0 = d_sslot + B;
    float *x = c->px.as<float>();
    uint16_t *xh = c->pxh.as<uint16_t>();
    const bool q8 = m->q8;
    if (q8 && (rc = ensure_q8(c, rows, std::max(H, std::max(QD, F)), std::max(H, std::max(QD, F))))) return rc;
    float *x32 = q8 ? c->x32.as<float>() : nullptr;
    launch_embed(c->pids.as<int32_t>(), rows, m->embd, H, d_feats, d_aud, x, s);
    const size_t layer_kv = (size_t)c->max_batch * hp.n_kv_head * c->max_ctx * 128;
    for (int l = 0; l < hp.dec_layers; l++) {
        const DecLayer &L = m->dec[l];
        launch_rmsnorm_f16(x, H, nullptr, rows, H, L.attn_norm, hp.rms_eps, xh, s, x32);
        GemmArgs q{};
        q.M = rows; q.N = QD + 2 * KD; q.K = H; q.out_f32 = c->pqkv.as<float>(); q.ldo = QD + 2 * KD;
        if (q8) gemm_q8(c, EPI_F32, q, x32, nullptr, H, 0, L.wqkv, L.wqkv_d, s);
        else { q.A = xh; q.lda = H; q.W = L.wqkv; q.ldw = H; launch_gemm_c(c, AM_DENSE, EPI_F32, q, s); }
        QkvPostArgs qa{};
        qa.qkv = c->pqkv.as<float>(); qa.rows = rows; qa.row_seq = d_seq; qa.row_pos = d_pos;
        qa.q_norm = L.q_norm; qa.k_norm = L.k_norm; qa.eps = hp.rms_eps; qa.rope = c->rope;
        qa.n_head = hp.n_head; qa.n_kv_head = hp.n_kv_head; qa.q_out = c->pq.as<uint16_t>();
        qa.kc = c->kc + l * layer_kv; qa.vc = c->vc + l * layer_kv; qa.max_ctx = c->max_ctx;
        qa.vt = c->vt + l * layer_vt(c);
        if (al) { qa.q32 = c->pq32.as<float>(); qa.k32 = c->pk32.as<float>(); }
        launch_qkv_post(qa, s);
        PrefillAttnArgs pa{};
        pa.q = c->pq.as<uint16_t>(); pa.kc = qa.kc; pa.vc = qa.vc; pa.seq_row0 = d_srow0; pa.seq_len = d_slen;
        pa.seq_slot = d_sslot; pa.n_seq = B; pa.max_len = maxp; pa.n_head = hp.n_head; pa.n_kv_head = hp.n_kv_head;
        pa.max_ctx = c->max_ctx; pa.scale = 1.0f / sqrtf(128.0f); pa.out = c->patt.as<uint16_t>(); pa.out32 = x32;
        if (al) { pa.q32 = qa.q32; pa.k32 = qa.k32; }
        if (pos0) pa.seq_pos0 = d_spos0;
        if (c->fuse.fa_exact_prefill || al) launch_prefill_attention_exact(pa, s);   // ggml CPU FA numerics
        else launch_prefill_attention(pa, s);
        GemmArgs o{};
        o.M = rows; o.N = H; o.K = QD; o.res = x; o.ldr = H; o.out_f32 = x; o.ldo = H;
        if (q8) gemm_q8(c, EPI_F32, o, x32, nullptr, QD, 0, L.wo, L.wo_d, s);
        else { o.A = c->patt.as<uint16_t>(); o.lda = QD; o.W = L.wo; o.ldw = QD; launch_gemm_c(c, AM_DENSE, EPI_F32, o, s); }
        launch_rmsnorm_f16(x, H, nullptr, rows, H, L.ffn_norm, hp.rms_eps, xh, s, x32);
        GemmArgs gu{};
        gu.M = rows; gu.N = 2 * F; gu.K = H;
        if (q8) {   // SwiGLU in fp32 (the down projection quantises it); x32 is free once quantised
            gu.out_f32 = x32; gu.ldo = F;
            gemm_q8(c, EPI_SWIGLU_F32, gu, x32, nullptr, H, 0, L.wgu, L.wgu_d, s);
        } else {
            gu.A = xh; gu.lda = H; gu.W = L.wgu; gu.ldw = H; gu.out_f16 = c->pact.as<uint16_t>(); gu.ldo16 = F;
            launch_gemm_c(c, AM_DENSE, EPI_SWIGLU_F16, gu, s);
        }
        GemmArgs dn{};
        dn.M = rows; dn.N = H; dn.K = F; dn.res = x; dn.ldr = H; dn.out_f32 = x; dn.ldo = H;
        if (q8) gemm_q8(c, EPI_F32, dn, x32, nullptr, F, 0, L.wd, L.wd_d, s);
        else { dn.A = c->pact.as<uint16_t>(); dn.lda = F; dn.W = L.wd; dn.ldw = F; launch_gemm_c(c, AM_DENSE, EPI_F32, dn, s); }
    }
    return declined_check("prefill");
}

// prefill (src/text_decoder.cpp:588-684): layers, then the LAST row of each
// sequence -> RMSNorm -> tied LM head + argmax (:564-572)
// slots: the KV-cache slot of each sequence (nullptr: sequence b -> slot b);
// the decode state (d_tok / d_pos / d_nkv) is written for entries 0..B-1
static int run_prefill(qasr_ctx *c, const std::vector<int32_t> &ids, const std::vector<int> &P, const float *d_feats,
                       const std::vector<int> &audio_pos, const std::vector<int> &N, bool want_logits,
                       const std::vector<int> *slots = nullptr, const std::vector<int> *pos0 = nullptr) {
    int rc;
    if ((rc = prefill_layers(c, ids, P, d_feats, audio_pos, N, slots, pos0))) return rc;
    // granule tags repeat across runs at the same positions: back to zero (no valid tag)
    HIPCHK(hipMemsetAsync(c->d_gran, 0, (size_t)(c->m->hp.n_head + 2 * c->m->hp.n_kv_head) * 128 * 8, c->st));
    HIPCHK(hipMemsetAsync(c->d_sgran, 0, (size_t)c->m->hp.n_head * sgran_ld(c->max_ctx) * 8, c->st));
    qasr_model *m = c->m;
    const Hparams &hp = m->hp;
    const int B = (int)P.size(), H = hp.hidden;
    hipStream_t s = c->st;
    float *x = c->px.as<float>();
    uint16_t *xl = c->d_xh;
    launch_rmsnorm_f16(x, H, c->plast.as<int>(), B, H, m->out_norm, hp.rms_eps, xl, s);
    launch_fill_u64(c->d_amax, B, 0ull, s);
    if (B <= 8) {
        GemvArgs gv{};
        gv.xh = xl; gv.ldxh = H; gv.W = m->embd; gv.K = H; gv.N = hp.vocab; gv.M = B;
        gv.out_f32 = want_logits ? c->d_logits : nullptr; gv.ldo = hp.vocab; gv.amax = c->d_amax;
        launch_gemv(EPI_ARGMAX, gv, s);
    } else {
        GemmArgs lm{};
        lm.A = xl; lm.lda = H; lm.W = m->embd; lm.ldw = H; lm.M = B; lm.N = hp.vocab; lm.K = H;
        lm.out_f32 = want_logits ? c->d_logits : nullptr; lm.ldo = hp.vocab; lm.amax = c->d_amax;
        launch_gemm_c(c, AM_DENSE, EPI_ARGMAX, lm, s);
    }
    HIPCHK(hipMemsetAsync(c->d_step, 0, 4, s));
    launch_argmax_finish(c->d_amax, B, c->d_tok, c->d_hist, c->hist_cap, c->d_step, s);
    launch_fill_u64(c->d_amax, B, 0ull, s);   // zero at rest for the decode graph
    // decode state: next position = P_b, n_kv = P_b + 1 (the fed token's own key included)
    std::vector<int> pos(B), nkv(B);
    for (int b = 0; b < B; b++) {
        pos[b] = (pos0 ? (*pos0)[b] : 0) + P[b];
        nkv[b] = pos[b] + 1;
    }
    HIPCHK(hipMemcpyAsync(c->d_pos, pos.data(), B * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_nkv, nkv.data(), B * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));   // pos/nkv host vectors go out of scope
    HIPCHK(hipGetLastError());
    return declined_check("prefill LM head");
}

// decode-batch projections: the weight-streaming skinny GEMM where it takes
// the shape, the tiled GEMM otherwise
static void dec_gemm(qasr_ctx *c, int epi, GemmArgs g, hipStream_t s) {
    g.no_skinny = !c->fuse.skinny;
    g.skinny_inflight = c->fuse.skinny_inf;
    g.wdef = c->fuse.skinny_wdef;
    if (launch_gemm_skinny(epi, g, s)) return;
    launch_gemm(AM_DENSE, epi, g, s);
}

// Launch groups of one decode step, in stream order (decoder cut at nl layers):
//   0          embedding gather (batches; batch <= 8 fuses it into layer 0)
//   1 + 2l     layer l: QKV projection + attention (+ o-projection when fused)
//   2 + 2l     layer l: o-projection (when separate) + FFN
//   1 + 2nl    final norm + LM head + argmax (+ bookkeeping at batch <= 8)
//   2 + 2nl    bookkeeping (batches)
// A step is emitted as the groups in [lo, hi): whole (graph replay), or split
// around one probed group that runs between HIP events.
struct StepRange {
    int lo, hi;
    bool in(int g) const { return g >= lo && g < hi; }
};
static constexpr StepRange kWholeStep{0, 1 << 30};
static int step_layers(const qasr_ctx *c) { return c->dbg_layers > 0 ? c->dbg_layers : c->m->hp.dec_layers; }

// one decode step for B sequences: token d_tok at position d_pos;
// splits: attention grid (64-key splits) covering the longest context of the step
// returns 0, or an error (a launch that declined its shape: nothing runs silently short)
static int decode_step_kernels(qasr_ctx *c, int B, bool want_logits, StepRange r, int splits) {
    qasr_model *m = c->m;
    const Hparams &hp = m->hp;
    const int H = hp.hidden, QD = hp.n_head * 128, KD = hp.n_kv_head * 128, F = hp.dec_ffn;
    hipStream_t s = c->st;
    float *x = c->d_x;
    const bool skinny = B <= 8;
    // decode batches: the LM head as one launch (lmhead.hip's shape conditions)
    const bool lmh_one = !skinny && B <= 128 && c->fuse.lmh && H == 1024 && hp.vocab % 16 == 0;
    const size_t layer_kv = (size_t)c->max_batch * hp.n_kv_head * c->max_ctx * 128;
    const int nl = step_layers(c);   // diagnostic layer cap
    // probed group (emitted alone): every launch in it folds its block times into one record
    unsigned long long *stamp = r.hi - r.lo == 1 ? c->cur_stamp : nullptr;
    if (r.in(0) && !skinny) launch_embed(c->d_tok, B, m->embd, H, nullptr, nullptr, x, s);
    const int skip = c->dev_skip;   // 0 unless built with -DQASR_DIAG_SKIP (QASR_DEV_SKIP): drop kernels to price them
    if (c->d_trace && r.in(0)) (void)hipMemsetAsync(c->d_trace, 0, 6 * 4096 * 8 * 8, s);
    for (int l = 0; l < nl; l++) {
        const bool ga = r.in(1 + 2 * l), gb = r.in(2 + 2 * l);
        if (!ga && !gb) continue;
        const DecLayer &L = m->dec[l];
        auto tr = [&](int k) -> unsigned long long * {
            return c->d_trace && l == c->trace_layer ? c->d_trace + (size_t)k * 4096 * 8 : nullptr;
        };
        const bool q8 = m->q8;
        DecodeAttnArgs da{};
        da.qkv = c->d_qkv; da.q_norm = L.q_norm; da.k_norm = L.k_norm; da.eps = hp.rms_eps; da.rope = c->rope;
        da.pos = c->d_pos; da.kc = c->kc + l * layer_kv; da.vc = c->vc + l * layer_kv; da.seq_slot = c->d_slot; da.B = B;
        da.vt = c->vt + l * layer_vt(c);
        da.n_head = hp.n_head; da.n_kv_head = hp.n_kv_head; da.max_ctx = c->max_ctx; da.max_splits = c->max_splits; da.grid_splits = splits;
        da.scale = 1.0f / sqrtf(128.0f); da.part = c->d_part; da.counter = c->d_counter; da.out = c->d_att;
        da.out32 = q8 && skinny ? c->d_att32 : nullptr;
        if (q8 && !skinny) { da.outq = c->d_q8a; da.outd = c->d_q8d; }
        da.trace = tr(1);
        da.qcnt = c->d_qcnt;
        da.spl1 = c->fuse.spl1;
        da.stream_blocks = !skinny && c->fuse.att_stream ? c->fuse.slots_stream : 0;
        da.spl_batch = c->fuse.att_spl;
        da.kv_nt = c->fuse.kv_nt;
        da.stamp = stamp;
        GemvArgs o{};
        if (skinny) {
            if (q8) { o.x = c->d_att32; o.ldx = QD; o.Wd = L.wo_d; }
            else { o.xh = c->d_att; o.ldxh = QD; }
            o.trace = tr(2);
            o.W = L.wo; o.K = QD; o.N = H; o.M = B; o.res = x; o.ldr = H; o.out_f32 = x; o.ldo = H;
            o.stamp = stamp;
        }
        GemvArgs q1{};   // batch-1 QKV projection, launched together with the attention when fusable
        if (skinny) {
            q1.x = x; q1.ldx = H; q1.norm_w = L.attn_norm; q1.eps = hp.rms_eps; q1.W = L.wqkv; q1.Wd = L.wqkv_d; q1.K = H;
            q1.N = QD + 2 * KD; q1.M = B; q1.out_f32 = c->d_qkv; q1.ldo = QD + 2 * KD;
            if (l == 0) { q1.embd_ids = c->d_tok; q1.embd = m->embd; q1.x_store = x; }   // fused embedding gather
            q1.trace = tr(0);
            q1.stamp = stamp;
        }
        GemvArgs gu{}, dn{};   // batch <= 8 FFN
        if (skinny) {
            gu.x = x; gu.ldx = H; gu.norm_w = L.ffn_norm; gu.eps = hp.rms_eps; gu.W = L.wgu; gu.Wd = L.wgu_d; gu.K = H; gu.N = F; gu.M = B;
            if (q8) { gu.out_f32 = c->d_act32; gu.ldo = F; }
            else { gu.out_f16 = c->d_act; gu.ldo16 = F; }
            gu.trace = tr(3);
            gu.stamp = stamp;
            if (q8) { dn.x = c->d_act32; dn.ldx = F; dn.Wd = L.wd_d; }
            else { dn.xh = c->d_act; dn.ldxh = F; }
            dn.W = L.wd; dn.K = F; dn.N = H; dn.M = B; dn.res = x; dn.ldr = H; dn.out_f32 = x; dn.ldo = H;
            dn.trace = tr(4);
            dn.stamp = stamp;
        }
        const bool exact = exact_decode(c);
        const bool fusable = skinny && B == 1 && !q8 && !skip;
        unsigned int *att_done = c->d_attdone + (size_t)l * 128;   // this layer's replicas
        if (fusable) da.att_done = att_done;
        if (fusable && exact && c->fuse.gran) {   // ggml's attention numerics as the fused launch's chain role
            da.fx = 1;
            da.sgran = c->d_sgran;
            da.gran = c->d_gran;   // (the fused decision needs the granule hand-off)
            da.layer = l;
        }
        unsigned int *fcnt = c->d_ffncnt + (size_t)l * 1024, *fcnt_next = c->d_ffncnt + (size_t)((l + 1) % nl) * 1024;
        // 0 = separate launches, 1 = QKV + attention in one launch, 2 = + o-projection.  ggml's numerics
        // in the fused launch need the granule hand-off (the chain role reads the new v from its granule):
        // without it the exact attention runs as separate launches, never as the fused fp32 split-K form
        const int fmode = fusable && (!exact || c->fuse.gran) ? launch_qkv_attention1(q1, da, &o, c->fuse, s, true) : 0;
        const bool o_fused = fmode >= 2;
        if (l == std::min(c->probe_layer, nl - 1)) c->probe_o_fused = o_fused;
        if (l == 0) {
            c->last_fmode = fmode;
            c->last_fx = fmode && da.fx;
            c->last_attn = fmode ? (da.fx ? 1 : 0) : -1;   // -1: set below by the separate path
        }
        if (ga) {
            if (l == nl - 1) c->qkv_in_gran = false;
            if (fmode) {
                if (c->fuse.gran) { da.gran = c->d_gran; da.layer = l; }
                if (l == nl - 1) c->qkv_in_gran = c->fuse.gran != 0;
                (void)launch_qkv_attention1(q1, da, &o, c->fuse, s, false);
            } else {
                if (skinny) {
                    if (!(skip & 1)) launch_gemv(EPI_F32, q1, s);
                } else {
                    GemmArgs q{};
                    q.M = B; q.N = QD + 2 * KD; q.K = H; q.out_f32 = c->d_qkv; q.ldo = QD + 2 * KD;
                    if (q8) {
                        launch_rmsnorm_q8(x, H, B, H, L.attn_norm, hp.rms_eps, c->d_q8n, c->d_q8nd, s);
                        gemm_q8_pre(c, EPI_F32, q, L.wqkv, L.wqkv_d, s, c->d_q8n, c->d_q8nd);
                    } else {
                        launch_rmsnorm_f16(x, H, nullptr, B, H, L.attn_norm, hp.rms_eps, c->d_xh, s);
                        q.A = c->d_xh; q.lda = H; q.W = L.wqkv; q.ldw = H; dec_gemm(c, EPI_F32, q, s);
                    }
                }
                da.att_done = nullptr;
                if (skip & 2) {
                } else if (exact) {   // ggml CPU FA numerics: scores by the splits, then the in-order chain
                    da.scores = c->d_scores;
                    da.fx_seq = c->fuse.fx_seq;
                    const bool one = launch_decode_attention_exact_seq(da, s);
                    if (!one) {
                        launch_decode_attention(da, s);
                        launch_decode_attention_exact(da, s);
                    }
                    if (l == 0) c->last_attn = one ? 2 : 3;
                } else {
                    launch_decode_attention(da, s);
                    if (l == 0) c->last_attn = 0;
                }
            }
        }
        if (!gb) continue;
        if (skinny) {
            if (!o_fused && !(skip & 4)) launch_gemv(EPI_F32, o, s);
            if (o_fused) dn.zero8 = att_done;   // re-arm the fused o-proj's arrival counters
            if (skip & 24 || nl < 2 || !launch_ffn1(gu, dn, fcnt, fcnt_next, c->fuse, s)) {
                if (!(skip & 8)) launch_gemv(q8 ? EPI_SWIGLU_F32 : EPI_SWIGLU_F16, gu, s);
                if (!(skip & 16)) launch_gemv(EPI_F32, dn, s);
                else if (o_fused) (void)hipMemsetAsync(att_done, 0, 8 * 16 * 4, s);   // the skipped down-proj re-arms these
            }
        } else if (q8) {
            GemmArgs ob{};
            ob.M = B; ob.N = H; ob.K = QD; ob.res = x; ob.ldr = H; ob.out_f32 = x; ob.ldo = H;
            gemm_q8_pre(c, EPI_F32, ob, L.wo, L.wo_d, s);
            launch_rmsnorm_q8(x, H, B, H, L.ffn_norm, hp.rms_eps, c->d_q8n, c->d_q8nd, s);
            GemmArgs gu{};
            gu.M = B; gu.N = 2 * F; gu.K = H; gu.out_f32 = c->d_x32; gu.ldo = F;
            GemmArgs dn{};
            dn.M = B; dn.N = H; dn.K = F; dn.res = x; dn.ldr = H; dn.out_f32 = x; dn.ldo = H;
            // the down projection's Q8_0 input quantised in the gate/up epilogue (one launch
            // fewer a layer, the same bits); the two-launch form where the skinny GEMM declines
            if (gemm_q8_pre_swiglu_q8(c, gu, L.wgu, L.wgu_d, s, c->d_q8n, c->d_q8nd, c->d_q8a, c->d_q8d)) {
                gemm_q8_pre(c, EPI_F32, dn, L.wd, L.wd_d, s, c->d_q8a, c->d_q8d);
            } else {
                gemm_q8_pre(c, EPI_SWIGLU_F32, gu, L.wgu, L.wgu_d, s, c->d_q8n, c->d_q8nd);
                gemm_q8(c, EPI_F32, dn, c->d_x32, nullptr, F, 0, L.wd, L.wd_d, s, c->d_q8a, c->d_q8d, true);
            }
        } else {
            GemmArgs ob{};
            ob.A = c->d_att; ob.lda = QD; ob.W = L.wo; ob.ldw = QD; ob.M = B; ob.N = H; ob.K = QD; ob.res = x; ob.ldr = H; ob.out_f32 = x; ob.ldo = H;
            dec_gemm(c, EPI_F32, ob, s);
            launch_rmsnorm_f16(x, H, nullptr, B, H, L.ffn_norm, hp.rms_eps, c->d_xh, s);
            GemmArgs gu{};
            gu.A = c->d_xh; gu.lda = H; gu.W = L.wgu; gu.ldw = H; gu.M = B; gu.N = 2 * F; gu.K = H; gu.out_f16 = c->d_act; gu.ldo16 = F;
            dec_gemm(c, EPI_SWIGLU_F16, gu, s);
            GemmArgs dn{};
            dn.A = c->d_act; dn.lda = F; dn.W = L.wd; dn.ldw = F; dn.M = B; dn.N = H; dn.K = F; dn.res = x; dn.ldr = H; dn.out_f32 = x; dn.ldo = H;
            dec_gemm(c, EPI_F32, dn, s);
        }
    }
    if (r.in(1 + 2 * nl)) {
        if (skinny) {   // amax / done are zero at rest: the LM head's last workgroup re-arms them
            GemvArgs lm{};
            lm.x = x; lm.ldx = H; lm.norm_w = m->out_norm; lm.eps = hp.rms_eps; lm.W = m->embd; lm.K = H; lm.N = hp.vocab; lm.M = B;
            lm.out_f32 = want_logits ? c->d_logits : nullptr; lm.ldo = hp.vocab; lm.amax = c->d_amax;
            lm.done = c->d_done; lm.tok_out = c->d_tok; lm.hist = c->d_hist; lm.hist_stride = c->hist_cap; lm.step = c->d_step;
            lm.pos = c->d_pos;
            lm.stamp = stamp;
            launch_gemv(EPI_ARGMAX, lm, s);
        } else if (lmh_one) {   // norm + GEMM + argmax + bookkeeping in one launch (lmhead.hip)
            GemvArgs lm{};
            lm.x = x; lm.ldx = H; lm.norm_w = m->out_norm; lm.eps = hp.rms_eps; lm.W = m->embd; lm.K = H; lm.N = hp.vocab; lm.M = B;
            lm.out_f32 = want_logits ? c->d_logits : nullptr; lm.ldo = hp.vocab; lm.amax = c->d_amax;
            lm.done = c->d_done; lm.tok_out = c->d_tok; lm.hist = c->d_hist; lm.hist_stride = c->hist_cap; lm.step = c->d_step;
            lm.pos = c->d_pos; lm.nkv = c->d_nkv;
            lm.stamp = stamp;
            if (!launch_lmhead_batch(lm, s))   // (lmh_one mirrors its shape conditions: never expected)
                return fail(QASR_ERR_STATE, "decode step: the batched LM head declined B = " + std::to_string(B));
        } else {
            launch_fill_u64(c->d_amax, B, 0ull, s);
            launch_rmsnorm_f16(x, H, nullptr, B, H, m->out_norm, hp.rms_eps, c->d_xh, s);
            GemmArgs lm{};
            lm.A = c->d_xh; lm.lda = H; lm.W = m->embd; lm.ldw = H; lm.M = B; lm.N = hp.vocab; lm.K = H;
            lm.out_f32 = want_logits ? c->d_logits : nullptr; lm.ldo = hp.vocab; lm.amax = c->d_amax;
            dec_gemm(c, EPI_ARGMAX, lm, s);
        }
    }
    if (r.in(2 + 2 * nl) && !skinny && !lmh_one) {   // bookkeeping (fused into the LM-head GEMV at batch <= 8)
        launch_step_advance(c->d_pos, c->d_nkv, c->d_step, B, s);
        launch_argmax_finish(c->d_amax, B, c->d_tok, c->d_hist, c->hist_cap, c->d_step, s);
        launch_fill_u64(c->d_amax, B, 0ull, s);   // re-arm (zero at rest)
    }
    return declined_check("decode step");
}

// Kernel probes (qasr_set_probe): HIP events on the context stream around one
// launch group of every decode step of qasr_run; the rest of the step replays
// as two graphs around it.
//   1 = LM head + argmax (group 1 + 2nl)
//   2 = layer probe_layer's QKV + attention (+ o-projection): at batch 1 the
//       fused qkv_attn1_kernel, the dominant kernel of the headline decode
//   3 = layer probe_layer's o-projection (if separate) + FFN: at batch 1 the
//       fused ffn1_kernel
//   4 = decode batches (9..128 rows): layer probe_layer's attention launch
//       alone (decode_attn_seq_kernel: the only launch of group 2's set that
//       records device stamps at these batches; its bytes are the K / V^T rows
//       of every sequence plus its q / output rows -- the utterance set's
//       dominant decode kernel, bench.py utterance_set.roofline)
static int probe_group(const qasr_ctx *c) {
    const int nl = step_layers(c), pl = std::min(c->probe_layer, nl - 1);
    return c->probe == 1 ? 1 + 2 * nl : (c->probe == 2 || c->probe == 4) ? 1 + 2 * pl : 2 + 2 * pl;
}

// algorithmic HBM bytes of one launch of the probed group at decode step k
// (SURVEY.md §8(d)): weights streamed once for the batch + each sequence's
// K/V rows of the layer (fp16, n_kv = P_b + k + 1 keys) + activations
static double probe_bytes(const qasr_ctx *c, int B, int k) {
    const Hparams &hp = c->m->hp;
    const double H = hp.hidden, QD = hp.n_head * 128.0, KD = hp.n_kv_head * 128.0, F = hp.dec_ffn;
    const double wb = c->m->q8 ? 34.0 / 32.0 : 2.0;   // bytes per linear weight (Q8_0 block: 34 B / 32)
    if (c->probe == 1) return (double)hp.vocab * H * 2 + B * H * 4 + B * 8.0;
    if (c->probe == 4) {   // the attention launch: K and V^T rows (fp16) + q / k / v rows (fp32) in + output (fp16) out
        double kv = 0;
        for (int b = 0; b < B; b++) kv += (double)(c->run_P[b] + k + 1) * KD * 2 * 2;
        return kv + B * (QD + 2 * KD) * 4 + B * QD * 2;
    }
    if (c->probe == 2) {
        double kv = 0;
        for (int b = 0; b < B; b++) kv += (double)(c->run_P[b] + k + 1) * KD * 2 * 2;
        const bool o_in = c->probe_o_fused;
        return (QD + 2 * KD) * H * wb + B * H * 4 + (o_in ? H * QD * wb + B * H * 8 : 0.0) + kv + B * (QD + 2 * KD) * 4;
    }
    return 3 * F * H * wb + (c->probe_o_fused ? 0.0 : H * QD * wb) + B * H * 4 * 3;
}

static int capture(qasr_ctx *c, int B, bool want_logits, StepRange r, int splits, hipGraphExec_t *out) {
    hipGraph_t gr;
    HIPCHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    const int rc = decode_step_kernels(c, B, want_logits, r, splits);
    HIPCHK(hipStreamEndCapture(c->st, &gr));
    if (rc) {
        (void)hipGraphDestroy(gr);
        return rc;
    }
    HIPCHK(hipGraphInstantiate(out, gr, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(gr));
    return 0;
}

// split-grid bucket for a step whose longest sequence feeds position `pos`
// (rounded up to 4 splits = 256 keys, so a run re-captures every 256 steps)
static int split_bucket(qasr_ctx *c, int pos) {
    const int need = (pos + 1 + decode_split_len() - 1) / decode_split_len();
    return std::min(c->max_splits, (need + 3) / 4 * 4);
}

// prepare decode graphs for batch B; base = longest prompt (step k feeds base + k)
static int decode_graph(qasr_ctx *c, int B, bool want_logits, int base) {
    const int pg = c->probe ? probe_group(c) : -1;
    // (graphs are kept per (batch, split bucket): a stream's decode chunks switch between live-prefix batches)
    if (c->graph_logits != want_logits || c->graph_probe_group != pg) c->drop_graphs();
    c->graph_B = B;
    c->graph_logits = want_logits;
    c->graph_base = base;
    c->graph_probe_group = pg;
    return 0;
}

static int step_graphs(qasr_ctx *c, int splits, qasr_ctx::StepGraphs **out) {
    const int B = c->graph_B;
    auto &gs = c->graphs[B * 65536 + splits];
    int rc;
    if (!gs.full && (rc = capture(c, B, c->graph_logits, kWholeStep, splits, &gs.full))) return rc;
    if (c->probe && !gs.pre) {
        const int g = c->graph_probe_group;
        if ((rc = capture(c, B, c->graph_logits, StepRange{0, g}, splits, &gs.pre)) ||
            (rc = capture(c, B, c->graph_logits, StepRange{g + 1, 1 << 30}, splits, &gs.post)))
            return rc;
    }
    *out = &gs;
    return 0;
}

// one greedy step (k = 0-based step of the run); under a probe the probed
// group runs eagerly between HIP events
static int launch_step(qasr_ctx *c, int B, int k) {
    const int splits = split_bucket(c, c->graph_base + k);
    qasr_ctx::StepGraphs *gs = nullptr;
    int rc;
    if (!c->eager && (rc = step_graphs(c, splits, &gs))) return rc;
    if (!c->probe || k % c->probe_stride != 0) {
        if (c->eager) return decode_step_kernels(c, B, c->graph_logits, kWholeStep, splits);
        HIPCHK(hipGraphLaunch(gs->full, c->st));
        return 0;
    }
    while ((int)c->pev.size() < 2 * (k + 1)) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        c->pev.push_back(e);
    }
    const int g = c->graph_probe_group;
    if (c->eager) {
        if ((rc = decode_step_kernels(c, B, c->graph_logits, StepRange{0, g}, splits))) return rc;
    } else {
        HIPCHK(hipGraphLaunch(gs->pre, c->st));
    }
    HIPCHK(hipEventRecord(c->pev[2 * k], c->st));
    c->cur_stamp = k < c->max_ctx ? c->d_pstamp + (size_t)k * kStampRec : nullptr;
    rc = decode_step_kernels(c, B, c->graph_logits, StepRange{g, g + 1}, splits);
    c->cur_stamp = nullptr;
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->pev[2 * k + 1], c->st));
    if (c->eager) {
        if ((rc = decode_step_kernels(c, B, c->graph_logits, StepRange{g + 1, 1 << 30}, splits))) return rc;
    } else {
        HIPCHK(hipGraphLaunch(gs->post, c->st));
    }
    return 0;
}

// arm the device-clock records of a run's probed launches (qasr_run): per
// step kStampRec u64, starts (~0) then ends (0), one 256-B line per shard
static int probe_arm(qasr_ctx *c, int nsteps) {
    if (!c->probe || nsteps <= 0) return 0;
    const int n = std::min(nsteps, c->max_ctx);
    launch_fill_u64(c->d_pstamp, n * kStampRec, ~0ull, c->st);
    HIPCHK(hipMemset2DAsync(c->d_pstamp + STAMP_ENDS, kStampRec * 8, 0, STAMP_ENDS * 8, n, c->st));
    return 0;
}

static int probe_collect(qasr_ctx *c, int B, int nsteps) {
    if (!c->probe) return 0;
    const int n = std::min(nsteps, c->max_ctx);
    // the first word of every shard line: [step][64]
    std::vector<unsigned long long> st((size_t)n * 64);
    if (n > 0)
        HIPCHK(hipMemcpy2D(st.data(), 8, c->d_pstamp, 32 * 8, 8, (size_t)n * 64, hipMemcpyDeviceToHost));
    for (int k = 0; k < n; k++) {   // first block start -> last block end, 100 MHz clock
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int i = 0; i < 32; i++) { t0 = std::min(t0, st[(size_t)k * 64 + i]); t1 = std::max(t1, st[(size_t)k * 64 + 32 + i]); }
        if (t0 == ~0ull || t1 <= t0) continue;   // launches without records (batch > 8 groups)
        c->probe_dev_ms += (double)(t1 - t0) * 1e-5;
        c->probe_dev_n++;
    }
    for (int k = 0; k < nsteps; k += c->probe_stride) {   // (steps between strides left no records)
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, c->pev[2 * k], c->pev[2 * k + 1]));
        c->probe_ms += ms;
        c->probe_n++;
        c->probe_bytes += probe_bytes(c, B, k);
    }
    return 0;
}

extern "C" int qasr_set_probe(qasr_ctx *c, int kernel) {
    if (!c || kernel < 0 || kernel > 4) return fail(QASR_ERR_ARG, "bad probe id");
    c->probe = kernel;
    c->probe_ms = 0.0;
    c->probe_n = 0;
    c->probe_bytes = 0.0;
    c->probe_dev_ms = 0.0;
    c->probe_dev_n = 0;
    return 0;
}

extern "C" int qasr_get_probe_device(qasr_ctx *c, double *total_ms, int64_t *launches) {
    if (!c) return fail(QASR_ERR_ARG, "null context");
    if (total_ms) *total_ms = c->probe_dev_ms;
    if (launches) *launches = c->probe_dev_n;
    return 0;
}

extern "C" int qasr_get_probe(qasr_ctx *c, double *total_ms, int64_t *launches, double *bytes_per_launch) {
    if (!c) return fail(QASR_ERR_ARG, "null context");
    if (total_ms) *total_ms = c->probe_ms;
    if (launches) *launches = c->probe_n;
    if (bytes_per_launch) *bytes_per_launch = c->probe_n ? c->probe_bytes / c->probe_n : 0.0;
    return 0;
}

// ================================================================== C-ABI
extern "C" int qasr_mel(qasr_ctx *c, const float *const *pcm, const int *n, int B, float *mel_out) {
    if (!c || !pcm || !n || B <= 0 || !mel_out) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(c->m->device));
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    std::vector<long> off(B);
    std::vector<int> nn(n, n + B);
    long tot = 0;
    for (int b = 0; b < B; b++) { if (n[b] < 0) return fail(QASR_ERR_ARG, "negative length"); off[b] = tot; tot += n[b]; }
    int rc = ensure(c, c->pcm, std::max<long>(tot, 1) * 4);
    if (rc) return rc;
    for (int b = 0; b < B; b++)
        if (n[b]) HIPCHK(hipMemcpyAsync(c->pcm.as<float>() + off[b], pcm[b], (size_t)n[b] * 4, hipMemcpyHostToDevice, c->st));
    std::vector<long> mo;
    std::vector<int> T;
    if ((rc = run_mel(c, off, nn, mo, T))) return rc;
    long total = 0;
    for (int b = 0; b < B; b++) total += 128L * T[b];
    if (total) HIPCHK(hipMemcpyAsync(mel_out, c->mel.p, total * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// ---------------------------------------------------- standalone log-mel
// log_mel_spectrogram of the component API (include/mel_spectrogram.h,
// src/mel_spectrogram.h:53-55) takes no model: an engine holds the DFT /
// window tables and a filterbank on one device and runs the same mel kernels
// as a context (launch_mel, csrc/mel.hip).
struct qasr_mel_engine {
    int device = 0;
    hipStream_t st = nullptr;
    double2 *tw = nullptr;
    double *hann = nullptr;
    float *filt = nullptr;        // [128][201], the last filterbank run with
    std::vector<float> filt_host; // ... its host copy (re-uploaded when a call brings other values)
    float *pcm = nullptr, *out = nullptr;
    double *tmp = nullptr;
    unsigned long long *cmax = nullptr;
    MelClip *clip = nullptr;
    int2 *blocks = nullptr;
    size_t pcm_cap = 0, out_cap = 0, tmp_cap = 0, blk_cap = 0;
    ~qasr_mel_engine() {
        (void)hipSetDevice(device);
        for (void *p : {(void *)tw, (void *)hann, (void *)filt, (void *)pcm, (void *)out, (void *)tmp, (void *)cmax, (void *)clip,
                        (void *)blocks})
            if (p) (void)hipFree(p);
        if (st) (void)hipStreamDestroy(st);
    }
};

static int grow(void **p, size_t &cap, size_t bytes) {
    if (bytes <= cap && *p) return 0;
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    cap = std::max<size_t>(bytes + bytes / 4, 4096);
    HIPCHK(hipMalloc(p, cap));
    return 0;
}

extern "C" int qasr_mel_filters(float *out) {
    if (!out) return fail(QASR_ERR_ARG, "bad arguments");
    std::vector<float> f;
    mel_filters(f);
    memcpy(out, f.data(), f.size() * 4);
    return 0;
}

extern "C" int qasr_mel_engine_create(int device, qasr_mel_engine **out) {
    if (!out) return fail(QASR_ERR_ARG, "bad arguments");
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return fail(QASR_ERR_DEVICE, "no such HIP device");
    std::unique_ptr<qasr_mel_engine> e(new qasr_mel_engine());
    e->device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
    std::vector<double> tw, hn;
    dft_twiddles(tw);
    hann_window(hn);
    mel_filters(e->filt_host);
    HIPCHK(hipMalloc((void **)&e->tw, tw.size() * 8));
    HIPCHK(hipMalloc((void **)&e->hann, hn.size() * 8));
    HIPCHK(hipMalloc((void **)&e->filt, e->filt_host.size() * 4));
    HIPCHK(hipMalloc((void **)&e->cmax, 8));
    HIPCHK(hipMalloc((void **)&e->clip, sizeof(MelClip)));
    HIPCHK(hipMemcpy(e->tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->hann, hn.data(), hn.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->filt, e->filt_host.data(), e->filt_host.size() * 4, hipMemcpyHostToDevice));
    *out = e.release();
    return 0;
}

extern "C" void qasr_mel_engine_free(qasr_mel_engine *e) { delete e; }

extern "C" int qasr_mel_engine_run(qasr_mel_engine *e, const float *pcm, int n, const float *filters, float *mel_out) {
    if (!e || n < 0 || (n > 0 && !pcm) || (mel_frames(n) > 0 && !mel_out)) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(e->device));
    const int TF = n / 160 + 1, T = TF - 1;
    if (filters && memcmp(filters, e->filt_host.data(), e->filt_host.size() * 4) != 0) {
        memcpy(e->filt_host.data(), filters, e->filt_host.size() * 4);
        HIPCHK(hipMemcpyAsync(e->filt, e->filt_host.data(), e->filt_host.size() * 4, hipMemcpyHostToDevice, e->st));
    }
    std::vector<int2> blocks;
    for (int f = 0; f < TF; f += mel_frames_per_block()) blocks.push_back(make_int2(0, f));
    const MelClip clip{0, n, TF, 0, 0};
    int rc;
    if ((rc = grow((void **)&e->pcm, e->pcm_cap, std::max<size_t>((size_t)n, 1) * 4)) ||
        (rc = grow((void **)&e->tmp, e->tmp_cap, (size_t)128 * TF * 8)) ||
        (rc = grow((void **)&e->out, e->out_cap, std::max<size_t>((size_t)128 * T, 1) * 4)) ||
        (rc = grow((void **)&e->blocks, e->blk_cap, blocks.size() * sizeof(int2))))
        return rc;
    if (n) HIPCHK(hipMemcpyAsync(e->pcm, pcm, (size_t)n * 4, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->clip, &clip, sizeof clip, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->blocks, blocks.data(), blocks.size() * sizeof(int2), hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemsetAsync(e->cmax, 0, 8, e->st));
    launch_mel(e->pcm, e->clip, 1, e->blocks, (int)blocks.size(), e->tw, e->hann, e->filt, e->tmp, e->cmax, e->out, e->st);
    HIPCHK(hipGetLastError());
    if (T > 0) HIPCHK(hipMemcpyAsync(mel_out, e->out, (size_t)128 * T * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));   // (the host vectors above go out of scope)
    return 0;
}

static int encode_common(qasr_ctx *c, const float *mel, const int *T, int B, float *outp, bool conv_only, bool no_chunk = false) {
    if (!c || !mel || !T || B <= 0 || !outp) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(c->m->device));
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    std::vector<int> Tv(T, T + B);
    std::vector<long> mo(B);
    long tot = 0;
    for (int b = 0; b < B; b++) { if (T[b] < 0) return fail(QASR_ERR_ARG, "negative length"); mo[b] = tot; tot += 128L * T[b]; }
    int rc = ensure(c, c->mel, std::max<long>(tot, 1) * 4);
    if (rc) return rc;
    if (tot) HIPCHK(hipMemcpyAsync(c->mel.p, mel, tot * 4, hipMemcpyHostToDevice, c->st));
    std::vector<int> Nb;
    if ((rc = run_encoder(c, c->mel.as<float>(), mo, Tv, conv_only, Nb, no_chunk))) return rc;
    long N = 0;
    for (int v : Nb) N += v;
    const int width = conv_only ? c->m->hp.d_model : c->m->hp.hidden;
    if (N) HIPCHK(hipMemcpyAsync(outp, conv_only ? c->ex.p : c->feats.p, (size_t)N * width * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

extern "C" int qasr_encode(qasr_ctx *c, const float *mel, const int *T, int B, float *feats) {
    return encode_common(c, mel, T, B, feats, false);
}
extern "C" int qasr_encode_conv(qasr_ctx *c, const float *mel, const int *T, int B, float *out) {
    return encode_common(c, mel, T, B, out, true);
}
extern "C" int qasr_encode_no_chunk(qasr_ctx *c, const float *mel, const int *T, int B, float *feats) {
    return encode_common(c, mel, T, B, feats, false, true);
}
extern "C" int qasr_encoder_frames_no_chunk(int n_mel_frames) {
    int L = n_mel_frames;
    if (L <= 0) return 0;
    for (int i = 0; i < 3; i++) L = (L - 1) / 2 + 1;   // src/audio_encoder.cpp:304-310 over the whole length
    return L;
}

extern "C" int qasr_prefill(qasr_ctx *c, const int32_t *ids, const int *P, const float *feats, const int *audio_pos,
                            const int *N, int B, float *logits_last, int32_t *argmax) {
    if (!c || !ids || !P || B <= 0) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(c->m->device));
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    const int H = c->m->hp.hidden;
    std::vector<int> Pv(P, P + B), Nv(B, 0), ap(B, -1);
    long nid = 0, nf = 0;
    for (int b = 0; b < B; b++) {
        nid += P[b];
        if (feats && N) { Nv[b] = N[b]; nf += N[b]; }
        if (audio_pos) ap[b] = audio_pos[b];
    }
    for (long i = 0; i < nid; i++)
        if (ids[i] < 0 || ids[i] >= c->m->hp.vocab) return fail(QASR_ERR_ARG, "token id out of range");
    std::vector<int32_t> idv(ids, ids + nid);
    int rc;
    if (nf) {
        if ((rc = ensure(c, c->feats, (size_t)nf * H * 4))) return rc;
        HIPCHK(hipMemcpyAsync(c->feats.p, feats, (size_t)nf * H * 4, hipMemcpyHostToDevice, c->st));
    }
    if ((rc = run_prefill(c, idv, Pv, nf ? c->feats.as<float>() : nullptr, ap, Nv, logits_last != nullptr))) return rc;
    if (logits_last) HIPCHK(hipMemcpyAsync(logits_last, c->d_logits, (size_t)B * c->m->hp.vocab * 4, hipMemcpyDeviceToHost, c->st));
    if (argmax) HIPCHK(hipMemcpyAsync(argmax, c->d_tok, B * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// TextDecoder::forward with n_tokens > 1 at n_past > 0 (src/text_decoder.cpp:
// 392-581 builds one graph for the chunk): the chunk's rows through the
// prefill layers at positions n_past[b] .. n_past[b] + P[b] - 1, causal
// attention over the cached keys and the chunk's own; logits of each chunk's
// last row.  n_past[b] = 0 is the plain prefill.  With feats: forward_with_audio
// at any n_past (src/text_decoder.cpp:588-644, the splice of :431-459) -- rows
// [audio_pos[b], audio_pos[b] + N[b]) of the chunk take the audio embeddings
// when they fit inside it, as the reference's condition.
static int prefill_chunk_common(qasr_ctx *c, const int32_t *ids, const int *P, const int *n_past, const float *feats,
                                const int *audio_pos, const int *N, int B, float *logits_last, int32_t *argmax) {
    if (!c || !ids || !P || !n_past || B <= 0) return fail(QASR_ERR_ARG, "bad arguments");
    if (feats && (!N || !audio_pos)) return fail(QASR_ERR_ARG, "audio features need N and audio_pos");
    for (int b = 0; b < B; b++)
        if (P[b] < 0 || n_past[b] < 0 || (feats && N[b] < 0)) return fail(QASR_ERR_ARG, "negative P / n_past / N");
    HIPCHK(hipSetDevice(c->m->device));
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    const int H = c->m->hp.hidden;
    std::vector<int> Pv(P, P + B), Nv(B, 0), ap(B, -1), p0(n_past, n_past + B);
    long nid = 0, nf = 0;
    for (int b = 0; b < B; b++) {
        nid += P[b];
        if (feats && N) { Nv[b] = N[b]; nf += N[b]; }
        if (audio_pos) ap[b] = audio_pos[b];
    }
    for (long i = 0; i < nid; i++)
        if (ids[i] < 0 || ids[i] >= c->m->hp.vocab) return fail(QASR_ERR_ARG, "token id out of range");
    std::vector<int32_t> idv(ids, ids + nid);
    int rc;
    if (nf) {
        if ((rc = ensure(c, c->feats, (size_t)nf * H * 4))) return rc;
        HIPCHK(hipMemcpyAsync(c->feats.p, feats, (size_t)nf * H * 4, hipMemcpyHostToDevice, c->st));
    }
    if ((rc = run_prefill(c, idv, Pv, nf ? c->feats.as<float>() : nullptr, ap, Nv, logits_last != nullptr, nullptr, &p0)))
        return rc;
    if (logits_last) HIPCHK(hipMemcpyAsync(logits_last, c->d_logits, (size_t)B * c->m->hp.vocab * 4, hipMemcpyDeviceToHost, c->st));
    if (argmax) HIPCHK(hipMemcpyAsync(argmax, c->d_tok, B * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

extern "C" int qasr_prefill_chunk(qasr_ctx *c, const int32_t *ids, const int *P, const int *n_past, int B, float *logits_last,
                                  int32_t *argmax) {
    return prefill_chunk_common(c, ids, P, n_past, nullptr, nullptr, nullptr, B, logits_last, argmax);
}

extern "C" int qasr_prefill_chunk_audio(qasr_ctx *c, const int32_t *ids, const int *P, const int *n_past, const float *feats,
                                        const int *audio_pos, const int *N, int B, float *logits_last, int32_t *argmax) {
    return prefill_chunk_common(c, ids, P, n_past, feats, audio_pos, N, B, logits_last, argmax);
}

extern "C" int qasr_decode_step(qasr_ctx *c, const int32_t *tok, const int *n_past, int B, float *logits, int32_t *argmax) {
    if (!c || !tok || !n_past || B <= 0 || B > c->max_batch) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(c->m->device));
    // a caller may repeat a position (same tag): no granule of an earlier call may match
    HIPCHK(hipMemsetAsync(c->d_gran, 0, (size_t)(c->m->hp.n_head + 2 * c->m->hp.n_kv_head) * 128 * 8, c->st));
    HIPCHK(hipMemsetAsync(c->d_sgran, 0, (size_t)c->m->hp.n_head * sgran_ld(c->max_ctx) * 8, c->st));
    std::vector<int> pos(B), nkv(B);
    for (int b = 0; b < B; b++) {
        if (n_past[b] < 0 || n_past[b] + 1 > c->max_ctx) return fail(QASR_ERR_ARG, "Context length exceeded");
        if (tok[b] < 0 || tok[b] >= c->m->hp.vocab) return fail(QASR_ERR_ARG, "token id out of range");
        pos[b] = n_past[b];
        nkv[b] = n_past[b] + 1;
    }
    std::unique_lock<std::mutex> dev_lk;
    if (takes_fused(c, B)) {
        dev_lk = std::unique_lock<std::mutex>(device_lock(c->m->device));
        if (int rc = reset_counters(c)) return rc;   // zero at rest whatever the previous call's launch modes were
    }
    HIPCHK(hipMemcpyAsync(c->d_tok, tok, B * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->d_pos, pos.data(), B * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->d_nkv, nkv.data(), B * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemsetAsync(c->d_step, 0, 4, c->st));
    if (int rc = decode_step_kernels(c, B, logits != nullptr, kWholeStep, split_bucket(c, *std::max_element(pos.begin(), pos.end()))))
        return rc;
    HIPCHK(hipGetLastError());
    if (logits) HIPCHK(hipMemcpyAsync(logits, c->d_logits, (size_t)B * c->m->hp.vocab * 4, hipMemcpyDeviceToHost, c->st));
    if (argmax) HIPCHK(hipMemcpyAsync(argmax, c->d_tok, B * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return check_dev_err(c);
}

extern "C" int qasr_stage_audio(qasr_ctx *c, const float *const *pcm, const int *n, int B) {
    if (!c || !pcm || !n || B <= 0) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(c->m->device));
    c->staged_n.assign(n, n + B);
    c->staged_off.assign(B, 0);
    long tot = 0;
    for (int b = 0; b < B; b++) { if (n[b] < 0) return fail(QASR_ERR_ARG, "negative length"); c->staged_off[b] = tot; tot += n[b]; }
    int rc = ensure(c, c->pcm, std::max<long>(tot, 1) * 4);
    if (rc) return rc;
    for (int b = 0; b < B; b++)
        if (n[b]) HIPCHK(hipMemcpyAsync(c->pcm.as<float>() + c->staged_off[b], pcm[b], (size_t)n[b] * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

extern "C" int qasr_run(qasr_ctx *c, int max_tokens, int ignore_eos, int32_t *tokens, int *n_tokens, qasr_timings *t) {
    if (!c || max_tokens <= 0 || !tokens || !n_tokens) return fail(QASR_ERR_ARG, "bad arguments");
    const int B = (int)c->staged_n.size();
    if (B == 0) return fail(QASR_ERR_STATE, "no staged audio");
    if (B > c->max_batch) return fail(QASR_ERR_ARG, "staged clips exceed the context's max_batch (qasr_run_staged runs subsets)");
    HIPCHK(hipSetDevice(c->m->device));
    std::unique_lock<std::mutex> dev_lk;
    if (takes_fused(c, B)) {
        dev_lk = std::unique_lock<std::mutex>(device_lock(c->m->device));
        // the fused launches re-arm the next layer's counters as they go; within
        // a run the launch mode only moves from fused to separate (longer
        // contexts), so zero them once here, whatever the previous run left
        if (int rc = reset_counters(c)) return rc;
    }
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    qasr_model *m = c->m;
    const Hparams &hp = m->hp;
    hipStream_t s = c->st;
    RoctxRange run_range("qasr.run");   // host-side ranges for rocprofv3 --marker-trace
    HIPCHK(hipEventRecord(c->ev[0], s));
    std::vector<long> mo;
    std::vector<int> T;
    int rc;
    if ((rc = run_mel(c, c->staged_off, c->staged_n, mo, T))) return rc;
    HIPCHK(hipEventRecord(c->ev[1], s));
    std::vector<int> Nb;
    if ((rc = run_encoder(c, c->mel.as<float>(), mo, T, false, Nb))) return rc;
    HIPCHK(hipEventRecord(c->ev[2], s));
    std::vector<int32_t> ids;
    std::vector<int> P(B), ap(B);
    for (int b = 0; b < B; b++) {
        std::vector<int32_t> p = build_prompt(hp, Nb[b], c->sys_ids, &ap[b]);
        if (ap[b] < 0) return fail(QASR_ERR_ARG, "No audio_pad token found in input sequence");
        P[b] = (int)p.size();
        if (P[b] + max_tokens > c->max_ctx) return fail(QASR_ERR_ARG, "Context length exceeded (prompt + max_tokens > max_ctx)");
        ids.insert(ids.end(), p.begin(), p.end());
    }
    if ((rc = run_prefill(c, ids, P, c->feats.as<float>(), ap, Nb, false))) return rc;
    HIPCHK(hipEventRecord(c->ev[3], s));
    // greedy loop (src/qwen3_asr.cpp:270-296): step k feeds token k at position P+k-1
    c->run_P = P;
    if ((rc = decode_graph(c, B, false, *std::max_element(P.begin(), P.end())))) return rc;
    if ((rc = probe_arm(c, max_tokens - 1))) return rc;
    std::vector<int32_t> hist((size_t)B * c->hist_cap);
    int steps = 0;
    std::optional<RoctxRange> dec_range(std::in_place, "qasr.decode");
    // profile: an event after every step (decode.token); k = 0-based step
    auto step = [&](int k) -> int {
        int r = launch_step(c, B, k);
        if (r || !c->profile_on) return r;
        while ((int)c->step_ev.size() <= k) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            c->step_ev.push_back(e);
        }
        HIPCHK(hipEventRecord(c->step_ev[k], s));
        return 0;
    };
    if (c->tok_cb) {
        // per-token callback (src/qwen3_asr.cpp:255-291): every token reaches
        // the host as it is produced -- one synchronisation per step
        std::vector<char> live(B, 1);
        std::vector<int32_t> tok(B);
        auto deliver = [&](int n_gen) -> int {
            HIPCHK(hipMemcpyAsync(tok.data(), c->d_tok, B * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            for (int b = 0; b < B; b++) {
                if (!live[b]) continue;
                c->tok_cb(c->tok_cb_user, b, n_gen, tok[b]);
                if (!ignore_eos && tok[b] == hp.eos_id) live[b] = 0;
            }
            return 0;
        };
        if ((rc = deliver(1))) return rc;
        int k = 1;
        for (; k < max_tokens && std::count(live.begin(), live.end(), 1) > 0; k++) {
            if ((rc = step(k - 1)) || (rc = deliver(k + 1))) return rc;
        }
        steps = k - 1;
        HIPCHK(hipMemcpyAsync(hist.data(), c->d_hist, hist.size() * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    } else if (ignore_eos) {
        for (int k = 1; k < max_tokens; k++)
            if ((rc = step(k - 1))) return rc;
        steps = max_tokens - 1;
        HIPCHK(hipMemcpyAsync(hist.data(), c->d_hist, hist.size() * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        const int chunk = 8;
        auto all_done = [&](int done) -> int {   // 1 = every sequence has emitted EOS
            if (hipMemcpyAsync(hist.data(), c->d_hist, hist.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -1;
            for (int b = 0; b < B; b++) {
                bool fin = false;
                for (int k = 0; k <= done && !fin; k++) fin = hist[(size_t)b * c->hist_cap + k] == hp.eos_id;
                if (!fin) return 0;
            }
            return 1;
        };
        int done = 0, st = 0;
        while (done + 1 < max_tokens && (st = all_done(done)) == 0) {
            const int todo = std::min(chunk, max_tokens - 1 - done);
            for (int k = 0; k < todo; k++)
                if ((rc = step(done + k))) return rc;
            done += todo;
        }
        if (st < 0) return fail(QASR_ERR_DEVICE, "device copy failed in decode loop");
        HIPCHK(hipMemcpyAsync(hist.data(), c->d_hist, hist.size() * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        steps = done;
    }
    dec_range.reset();
    HIPCHK(hipEventRecord(c->ev[4], s));
    HIPCHK(hipEventSynchronize(c->ev[4]));
    if ((rc = check_dev_err(c))) return rc;
    if ((rc = probe_collect(c, B, steps))) return rc;
    if (c->profile_on) {   // the reference's QWEN3_TIMER sections (src/timing.h), device time
        auto add = [&](const char *name, hipEvent_t e0, hipEvent_t e1) -> int {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, e0, e1));
            auto &v = c->prof[name];
            v.first += ms;
            v.second += 1;
            return 0;
        };
        if ((rc = add("mel_spectrogram", c->ev[0], c->ev[1])) || (rc = add("audio_encoding.total", c->ev[1], c->ev[2])) ||
            (rc = add("audio_encoding.conv_chunk", c->ev[1], c->ev[5])) ||
            (rc = add("audio_encoding.transformer", c->ev[5], c->ev[2])) ||
            (rc = add("decode.initial_forward", c->ev[2], c->ev[3])) || (rc = add("transcribe.total", c->ev[0], c->ev[4])))
            return rc;
        for (int k = 0; k < steps; k++)
            if ((rc = add("decode.token", k ? c->step_ev[k - 1] : c->ev[3], c->step_ev[k]))) return rc;
    }
    if (c->d_trace) {   // dev trace dump: raw [6][4096][8] u64
        std::vector<unsigned long long> tr((size_t)6 * 4096 * 8);
        HIPCHK(hipMemcpy(tr.data(), c->d_trace, tr.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = fopen(c->trace_path.c_str(), "wb")) {
            (void)fwrite(tr.data(), 8, tr.size(), f);
            fclose(f);
        }
    }
    for (int b = 0; b < B; b++) {
        int nt = 0;
        for (int k = 0; k <= steps && k < max_tokens; k++) {
            const int32_t tk = hist[(size_t)b * c->hist_cap + k];
            tokens[(size_t)b * max_tokens + nt++] = tk;
            if (!ignore_eos && tk == hp.eos_id) break;
        }
        if (!ignore_eos && nt > 0 && tokens[(size_t)b * max_tokens + nt - 1] == hp.eos_id) nt--;
        n_tokens[b] = nt;
    }
    if (t) {
        float a, b2, c2, d;
        (void)hipEventElapsedTime(&a, c->ev[0], c->ev[1]);
        (void)hipEventElapsedTime(&b2, c->ev[1], c->ev[2]);
        (void)hipEventElapsedTime(&c2, c->ev[2], c->ev[3]);
        (void)hipEventElapsedTime(&d, c->ev[3], c->ev[4]);
        t->t_mel_ms = a; t->t_encode_ms = b2; t->t_prefill_ms = c2; t->t_decode_ms = d;
        t->t_total_ms = (double)a + b2 + c2 + d;
        t->n_decode_steps = steps;
    }
    return 0;
}

extern "C" int qasr_run_staged(qasr_ctx *c, const int *clips, int B, int max_tokens, int ignore_eos, int32_t *tokens,
                               int *n_tokens, qasr_timings *t) {
    if (!c || !clips || B <= 0) return fail(QASR_ERR_ARG, "bad arguments");
    if (B > c->max_batch) return fail(QASR_ERR_ARG, "subset exceeds the context's max_batch");
    std::vector<int> n(B);
    std::vector<long> off(B);
    for (int b = 0; b < B; b++) {
        if (clips[b] < 0 || clips[b] >= (int)c->staged_n.size()) return fail(QASR_ERR_ARG, "staged clip index out of range");
        n[b] = c->staged_n[clips[b]];
        off[b] = c->staged_off[clips[b]];
    }
    std::swap(n, c->staged_n);
    std::swap(off, c->staged_off);
    const int rc = qasr_run(c, max_tokens, ignore_eos, tokens, n_tokens, t);
    std::swap(n, c->staged_n);   // the staged pool stays for the next subset
    std::swap(off, c->staged_off);
    return rc;
}

// ------------------------------------------------------ continuous batching
// qasr_run_stream: `slots` KV-cache slots (<= max_batch) decode together;
// a slot whose clip ends (EOS, or its token budget) is refilled at the next
// chunk boundary -- mel + encoder + prefill of the next clips from `fetch`
// into exactly the freed slots (prefill_layers' slot map), the other slots'
// caches untouched -- so a batch never idles on its longest member (the
// reference decodes one utterance at a time, src/qwen3_asr.cpp:270-296; the
// tokens of a clip depend only on its own rows).  Every chunk of <= 8 steps
// (1 with a token callback) replays the step graphs of qasr_run, then the
// host reads the chunk's tokens, delivers finished clips to `sink` and
// re-uploads the slots' (token, position) state.  A slot with no clip is
// parked at position 0 (its writes stay inside its own cache slot).
namespace {
struct StreamSlot {
    int id = -1, P = 0, budget = 0;
    std::vector<int32_t> toks;
};
}  // namespace

// next(clip) -> false when the queue is empty; a clip is host samples (pcm, n)
// or a clip of the staged pool (staged >= 0)
struct StreamClip {
    int id = -1, budget = 0, n = 0, staged = -1;
    const float *pcm = nullptr;
};
static int run_stream(qasr_ctx *c, int slots, const std::function<bool(StreamClip &)> &next, qasr_sink_fn sink, void *user,
                      int max_tokens, int ignore_eos, qasr_stream_stats *stats) {
    if (!c || !sink || max_tokens <= 0 || slots < 0 || slots > c->max_batch) return fail(QASR_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(c->m->device));
    const int S = slots ? slots : c->max_batch;
    std::unique_lock<std::mutex> dev_lk;
    if (takes_fused(c, S)) {
        dev_lk = std::unique_lock<std::mutex>(device_lock(c->m->device));
        if (int rc = reset_counters(c)) return rc;
    }
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    const Hparams &hp = c->m->hp;
    hipStream_t s = c->st;
    const auto t_start = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point t0) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    qasr_stream_stats st{};
    // device time of each refill's mel and encoder stages (the utterance set's encoder roofline)
    struct StageEvents {
        hipEvent_t e[3] = {nullptr, nullptr, nullptr};
        ~StageEvents() { for (hipEvent_t x : e) if (x) (void)hipEventDestroy(x); }
    } ev;
    for (hipEvent_t &x : ev.e) HIPCHK(hipEventCreate(&x));
    std::vector<StreamSlot> sl(S);
    bool open = true;
    int rc;
    // a finished clip: trailing EOS popped (src/qwen3_asr.cpp:298-300)
    auto deliver = [&](StreamSlot &x) {
        std::vector<int32_t> &t = x.toks;
        if (!ignore_eos && !t.empty() && t.back() == hp.eos_id) t.pop_back();
        sink(user, x.id, 0, t.data(), (int)t.size());
        st.n_clips++;
        x.id = -1;
        x.toks.clear();
    };
    auto reject = [&](int id, int code, const char *msg) {   // per-clip error: the message is qasr_last_error() inside sink
        fail(code, msg);
        sink(user, id, code, nullptr, 0);
        st.n_errors++;
    };
    // fill free slots from the queue until every slot holds a live clip or the queue is empty
    auto refill = [&]() -> int {
        bool refilled = false;
        for (;;) {
            std::vector<int> freeS;
            for (int i = 0; i < S; i++)
                if (sl[i].id < 0) freeS.push_back(i);
            if (freeS.empty() || !open) return 0;
            if (refilled && c->fuse.refill_group > 0) return 0;   // one group a refill: decode steps come between groups
            if (c->fuse.refill_group > 0 && (int)freeS.size() > c->fuse.refill_group) freeS.resize(c->fuse.refill_group);
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<int> ids, ns, budgets, slots;
            std::vector<float> pcm;   // host clips of this refill, packed (-> c->spcm)
            std::vector<long> off;
            bool staged = false;
            while (ids.size() < freeS.size()) {
                StreamClip k;
                k.budget = max_tokens;
                if (!next(k)) { open = false; break; }
                const int id = k.id;
                if (k.staged >= 0) {
                    if (k.staged >= (int)c->staged_n.size()) { reject(id, QASR_ERR_ARG, "staged clip index out of range"); continue; }
                    k.n = c->staged_n[k.staged];
                }
                const int P = qasr_prompt_len(encoder_frames(mel_frames(std::max(k.n, 0)))) + (int)c->sys_ids.size();
                if (k.n < 0 || (k.staged < 0 && k.n > 0 && !k.pcm) || k.budget <= 0) { reject(id, QASR_ERR_ARG, "bad clip (length, samples or budget)"); continue; }
                if (encoder_frames(mel_frames(k.n)) <= 0) { reject(id, QASR_ERR_ARG, "No audio_pad token found in input sequence"); continue; }
                if (P + k.budget > c->max_ctx) { reject(id, QASR_ERR_ARG, "Context length exceeded (prompt + max_tokens > max_ctx)"); continue; }
                staged = k.staged >= 0;   // (one kind per run: the caller's API)
                ids.push_back(id);
                ns.push_back(k.n);
                budgets.push_back(k.budget);
                if (staged) {
                    off.push_back(c->staged_off[k.staged]);
                } else {
                    off.push_back((long)pcm.size());
                    pcm.insert(pcm.end(), k.pcm, k.pcm + k.n);
                }
                slots.push_back(freeS[ids.size() - 1]);
            }
            if (ids.empty()) return 0;
            const int R = (int)ids.size();
            if (!staged) {
                if ((rc = ensure(c, c->spcm, std::max<size_t>(pcm.size(), 1) * 4))) return rc;
                HIPCHK(hipMemcpyAsync(c->spcm.p, pcm.data(), pcm.size() * 4, hipMemcpyHostToDevice, s));
            }
            std::vector<long> mo;
            std::vector<int> T, Nb;
            HIPCHK(hipEventRecord(ev.e[0], s));
            if ((rc = run_mel(c, off, ns, mo, T, staged ? c->pcm.as<float>() : c->spcm.as<float>()))) return rc;
            HIPCHK(hipEventRecord(ev.e[1], s));
            if ((rc = run_encoder(c, c->mel.as<float>(), mo, T, false, Nb))) return rc;
            HIPCHK(hipEventRecord(ev.e[2], s));
            std::vector<int32_t> pids;
            std::vector<int> P(R), ap(R);
            for (int r = 0; r < R; r++) {
                std::vector<int32_t> pr = build_prompt(hp, Nb[r], c->sys_ids, &ap[r]);
                if (ap[r] < 0 || (int)pr.size() + budgets[r] > c->max_ctx) return fail(QASR_ERR_STATE, "prompt length differs from its estimate");
                P[r] = (int)pr.size();
                pids.insert(pids.end(), pr.begin(), pr.end());
            }
            if ((rc = run_prefill(c, pids, P, c->feats.as<float>(), ap, Nb, false, &slots))) return rc;
            std::vector<int32_t> first(R);
            HIPCHK(hipMemcpyAsync(first.data(), c->d_tok, R * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));   // (pcm host vector in flight until here)
            if ((rc = check_dev_err(c))) return rc;
            refilled = true;
            st.n_prefills++;
            st.t_prefill_ms += ms_since(t0);
            float mel_ms = 0.f, enc_ms = 0.f;
            HIPCHK(hipEventElapsedTime(&mel_ms, ev.e[0], ev.e[1]));
            HIPCHK(hipEventElapsedTime(&enc_ms, ev.e[1], ev.e[2]));
            st.t_mel_ms += mel_ms;
            st.t_encode_ms += enc_ms;
            for (int r = 0; r < R; r++) {
                StreamSlot &x = sl[slots[r]];
                x.id = ids[r];
                x.P = P[r];
                x.budget = budgets[r];
                x.toks.assign(1, first[r]);
                if (c->tok_cb) c->tok_cb(c->tok_cb_user, x.id, 1, first[r]);
                if ((!ignore_eos && first[r] == hp.eos_id) || x.budget == 1) deliver(x);
            }
        }
    };
    std::vector<int> pos(S), nkv(S), tok(S);
    std::vector<int32_t> hist;
    if ((rc = decode_graph(c, S, false, 0))) return rc;
    for (;;) {
        if ((rc = refill())) return rc;
        int live = 0, chunk = c->tok_cb ? 1 : 8, maxpos = 0, hi = 0;
        for (int i = 0; i < S; i++) {
            const StreamSlot &x = sl[i];
            if (x.id < 0) { pos[i] = 0; nkv[i] = 1; tok[i] = 0; continue; }   // parked
            live++;
            hi = i + 1;
            pos[i] = x.P + (int)x.toks.size() - 1;   // the last token is fed at this position
            nkv[i] = pos[i] + 1;
            tok[i] = x.toks.back();
            chunk = std::min(chunk, x.budget - (int)x.toks.size());
            maxpos = std::max(maxpos, pos[i]);
        }
        if (live == 0) break;
        // option live_prefix: decode only the slots up to the last live one (rounded up to 16 rows, at least
        // 16 -- the batch kernels' shapes), so a context filling in refill groups or draining at the end of the
        // queue does not run every step at full width; the slots past it are parked and untouched
        const int Bq = c->fuse.live_prefix && S > 8 ? std::min(S, std::max(16, (hi + 15) / 16 * 16)) : S;
        if ((rc = decode_graph(c, Bq, false, 0))) return rc;
        HIPCHK(hipMemcpyAsync(c->d_pos, pos.data(), S * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_nkv, nkv.data(), S * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_tok, tok.data(), S * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemsetAsync(c->d_step, 0, 4, s));
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < chunk; k++) {
            const int splits = split_bucket(c, maxpos + k);
            if (c->eager) {
                if ((rc = decode_step_kernels(c, Bq, false, kWholeStep, splits))) return rc;
            } else {
                qasr_ctx::StepGraphs *gs = nullptr;
                if ((rc = step_graphs(c, splits, &gs))) return rc;
                HIPCHK(hipGraphLaunch(gs->full, s));
            }
        }
        hist.resize((size_t)S * chunk);
        // (a decode step advances d_step, then writes hist[step]: the chunk's tokens are columns 1..chunk)
        HIPCHK(hipMemcpy2DAsync(hist.data(), chunk * 4, c->d_hist + 1, (size_t)c->hist_cap * 4, chunk * 4, S, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));   // (the pos / nkv / tok host vectors in flight until here)
        if ((rc = check_dev_err(c))) return rc;
        st.t_decode_ms += ms_since(t0);
        st.n_steps += chunk;
        st.slot_steps += (int64_t)S * chunk;
        for (int i = 0; i < S; i++) st.kv_keys += (int64_t)nkv[i] * chunk + (int64_t)chunk * (chunk - 1) / 2;   // step k: n_kv + k
        for (int i = 0; i < S; i++) {
            StreamSlot &x = sl[i];
            if (x.id < 0) continue;
            for (int k = 0; k < chunk; k++) {
                const int32_t t = hist[(size_t)i * chunk + k];
                x.toks.push_back(t);
                st.live_steps++;
                if (c->tok_cb) c->tok_cb(c->tok_cb_user, x.id, (int)x.toks.size(), t);
                if ((!ignore_eos && t == hp.eos_id) || (int)x.toks.size() >= x.budget) {
                    deliver(x);
                    break;
                }
            }
        }
    }
    st.t_total_ms = ms_since(t_start);
    if (stats) *stats = st;
    return 0;
}

extern "C" int qasr_run_stream(qasr_ctx *c, int slots, qasr_fetch_fn fetch, qasr_sink_fn sink, void *user, int max_tokens,
                               int ignore_eos, qasr_stream_stats *stats) {
    if (!fetch) return fail(QASR_ERR_ARG, "bad arguments");
    return run_stream(c, slots, [&](StreamClip &k) { return (k.id = fetch(user, &k.pcm, &k.n, &k.budget)) >= 0; }, sink, user,
                      max_tokens, ignore_eos, stats);
}

extern "C" int qasr_run_stream_staged(qasr_ctx *c, int slots, qasr_fetch_staged_fn fetch, qasr_sink_fn sink, void *user,
                                      int max_tokens, int ignore_eos, qasr_stream_stats *stats) {
    if (!fetch) return fail(QASR_ERR_ARG, "bad arguments");
    const int pool = (int)c->staged_n.size();
    return run_stream(c, slots, [&](StreamClip &k) {
        k.id = fetch(user, &k.budget);
        // ids past the pool reuse its clips only when asked for (option staged_wrap); else run_stream
        // rejects them as out of range
        k.staged = k.id >= 0 && pool > 0 && c->fuse.staged_wrap ? k.id % pool : k.id;
        return k.id >= 0;
    }, sink, user, max_tokens, ignore_eos, stats);
}

extern "C" int qasr_set_token_callback(qasr_ctx *c, void (*cb)(void *user, int seq, int n_generated, int32_t token), void *user) {
    if (!c) return fail(QASR_ERR_ARG, "null context");
    c->tok_cb = cb;
    c->tok_cb_user = user;
    return 0;
}

extern "C" int qasr_set_profile(qasr_ctx *c, int on) {
    if (!c) return fail(QASR_ERR_ARG, "null context");
    c->profile_on = on != 0;
    c->prof.clear();
    return 0;
}

// QWEN3_TIMER_REPORT's table (src/timing.h:32-48) over the sections recorded since qasr_set_profile
extern "C" int qasr_profile_report(qasr_ctx *c, char *out, int cap) {
    if (!c) return fail(QASR_ERR_ARG, "null context");
    std::string r = "\n================================================================================\n"
                    "                         TIMING PROFILE REPORT\n"
                    "================================================================================\n";
    char line[160];
    snprintf(line, sizeof line, "%-45s %12s %8s %12s\n", "Section", "Total (ms)", "Calls", "Avg (ms)");
    r += line;
    r += "--------------------------------------------------------------------------------\n";
    for (const auto &kv : c->prof) {
        snprintf(line, sizeof line, "%-45s %12.2f %8ld %12.2f\n", kv.first.c_str(), kv.second.first, kv.second.second,
                 kv.second.second ? kv.second.first / kv.second.second : 0.0);
        r += line;
    }
    r += "================================================================================\n";
    if (out && cap > 0) {
        const size_t n = std::min(r.size(), (size_t)cap - 1);
        memcpy(out, r.data(), n);
        out[n] = 0;
    }
    return (int)r.size();
}

extern "C" int qasr_set_system_prompt(qasr_ctx *c, const int32_t *ids, int n) {
    if (!c || n < 0 || (n > 0 && !ids)) return fail(QASR_ERR_ARG, "bad arguments");
    c->sys_ids.assign(ids, ids + n);
    return 0;
}

extern "C" int qasr_transcribe_batch(qasr_ctx *c, const float *const *pcm, const int *n, int B, int max_tokens, int ignore_eos,
                                     int32_t *tokens, int *n_tokens, qasr_timings *t) {
    int rc = qasr_stage_audio(c, pcm, n, B);
    if (rc) return rc;
    return qasr_run(c, max_tokens, ignore_eos, tokens, n_tokens, t);
}

// ------------------------------------------------------------------- text
extern "C" int qasr_detokenize(const qasr_model *m, const int32_t *ids, int n, char *out, int cap) {
    if (!m || (!ids && n > 0)) return fail(QASR_ERR_ARG, "bad arguments");
    std::string s = m->tok.decode(std::vector<int32_t>(ids, ids + n));
    if (out && cap > 0) {
        const int k = std::min<int>((int)s.size(), cap - 1);
        memcpy(out, s.data(), k);
        out[k] = 0;
    }
    return (int)s.size();
}

extern "C" int qasr_tokenize(const qasr_model *m, const char *text, int32_t *ids, int cap) {
    if (!m || !text) return fail(QASR_ERR_ARG, "bad arguments");
    std::vector<int32_t> v = m->tok.encode(text);
    if (ids) for (int i = 0; i < (int)v.size() && i < cap; i++) ids[i] = v[i];
    return (int)v.size();
}

// ------------------------------------------------------------ forced aligner
// ForcedAligner::align (src/forced_aligner.cpp:1636-1720), device part: mel ->
// aligner encoder (padded chunks, 104-frame windows) -> <|audio_start|> pad x n
// <|audio_end|> text prompt (n from HF _get_feat_extract_output_lengths, the
// encoder rows spliced from index 1) -> one causal prefill -> at every
// timestamp-token row: RMSNorm -> classify head -> argmax (strict '>', :1280-1306).
// B clips at once (configs[4]'s aligner leg over a rank's transcripts): the
// mel and the windowed encoder of all clips in one pass, one prefill of the B
// prompts (prefill_layers' sequences), one classify GEMM over every timestamp
// row of every clip.  Rows are independent in each of them, so a clip's
// classes are the same alone or in a batch (tests/test_gpu_aligner.py).
static int align_classes(qasr_ctx *c, const float *const *pcm, const int *n, const std::vector<std::vector<int32_t>> &text_ids,
                         std::vector<std::vector<int32_t>> &classes, qasr_timings *t) {
    qasr_model *m = c->m;
    const Hparams &hp = m->hp;
    const int B = (int)text_ids.size();
    if (!hp.aligner || !m->cls_w) return fail(QASR_ERR_STATE, "not a ForcedAligner model");
    if (B <= 0 || B > c->max_batch) return fail(QASR_ERR_ARG, "aligner batch exceeds the context's max_batch");
    HIPCHK(hipSetDevice(m->device));
    HIPCHK(hipStreamSynchronize(c->st));
    c->pin_used = 0;
    hipStream_t s = c->st;
    int rc;
    std::vector<long> off(B);
    std::vector<int> nv(n, n + B);
    long tot = 0;
    for (int b = 0; b < B; b++) {
        if (n[b] <= 0) return fail(QASR_ERR_ARG, "bad arguments");
        off[b] = tot;
        tot += n[b];
    }
    if ((rc = ensure(c, c->pcm, (size_t)std::max<long>(tot, 1) * 4))) return rc;
    for (int b = 0; b < B; b++)
        HIPCHK(hipMemcpyAsync(c->pcm.as<float>() + off[b], pcm[b], (size_t)n[b] * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(c->ev[0], s));
    std::vector<long> mo;
    std::vector<int> T, Nb;
    if ((rc = run_mel(c, off, nv, mo, T))) return rc;
    HIPCHK(hipEventRecord(c->ev[1], s));
    if ((rc = run_encoder(c, c->mel.as<float>(), mo, T, false, Nb))) return rc;
    HIPCHK(hipEventRecord(c->ev[2], s));
    std::vector<int32_t> ids;
    std::vector<int> P(B), ap(B, 1), rows, nrows(B, 0);
    for (int b = 0; b < B; b++) {
        const std::vector<int32_t> ib = build_align_tokens(hp, text_ids[b], feat_extract_output_lengths(T[b]));
        P[b] = (int)ib.size();
        if (P[b] > c->max_ctx) return fail(QASR_ERR_ARG, "Context length exceeded (aligner prompt > max_ctx)");
        for (int i = 0; i < P[b]; i++)
            if (ib[i] == hp.timestamp_id) {
                rows.push_back((int)ids.size() + i);   // the row in the prefill's concatenated rows
                nrows[b]++;
            }
        ids.insert(ids.end(), ib.begin(), ib.end());
    }
    if ((rc = prefill_layers(c, ids, P, c->feats.as<float>(), ap, Nb, nullptr))) return rc;
    const int NT = (int)rows.size(), H = hp.hidden;
    std::vector<unsigned long long> keys(NT);
    if (NT > 0) {
        if ((rc = upload(c, c->ats, rows)) || (rc = ensure(c, c->atx, (size_t)NT * H * 2)) || (rc = ensure(c, c->aam, (size_t)NT * 8)))
            return rc;
        HIPCHK(hipMemsetAsync(c->aam.p, 0, (size_t)NT * 8, s));
        launch_rmsnorm_f16(c->px.as<float>(), H, c->ats.as<int>(), NT, H, m->out_norm, hp.rms_eps, c->atx.as<uint16_t>(), s);
        GemmArgs g{};
        g.A = c->atx.as<uint16_t>(); g.lda = H; g.W = m->cls_w; g.ldw = H; g.M = NT; g.N = m->cls_rows; g.K = H;
        g.amax = c->aam.as<unsigned long long>(); g.n_valid = hp.classify_num;
        launch_gemm_c(c, AM_DENSE, EPI_ARGMAX, g, s);
        HIPCHK(hipGetLastError());
        if ((rc = declined_check("aligner head"))) return rc;
        HIPCHK(hipMemcpyAsync(keys.data(), c->aam.p, (size_t)NT * 8, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipEventRecord(c->ev[3], s));
    HIPCHK(hipEventSynchronize(c->ev[3]));
    classes.assign(B, {});
    for (int b = 0, k = 0; b < B; b++)
        for (int i = 0; i < nrows[b]; i++, k++) classes[b].push_back((int32_t)(0xffffffffu - (uint32_t)(keys[k] & 0xffffffffu)));
    if (t) {
        float a = 0, bb = 0, d = 0, tt = 0;
        HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
        HIPCHK(hipEventElapsedTime(&bb, c->ev[1], c->ev[2]));
        HIPCHK(hipEventElapsedTime(&d, c->ev[2], c->ev[3]));
        HIPCHK(hipEventElapsedTime(&tt, c->ev[0], c->ev[3]));
        *t = qasr_timings{a, bb, d, 0.0, tt, 0};
    }
    return 0;
}
static int align_classes(qasr_ctx *c, const float *pcm, int n, const std::vector<int32_t> &text_ids, std::vector<int32_t> &classes,
                         qasr_timings *t) {
    std::vector<std::vector<int32_t>> cls;
    const int rc = align_classes(c, &pcm, &n, {text_ids}, cls, t);
    if (!rc) classes = cls[0];
    return rc;
}

extern "C" int qasr_align(qasr_ctx *c, const float *pcm, int n, const int32_t *text_ids, int n_text, int32_t *classes,
                          int cap, int *n_ts, qasr_timings *t) {
    if (!c || !pcm || n <= 0 || n_text < 0 || (n_text && !text_ids) || !n_ts) return fail(QASR_ERR_ARG, "bad arguments");
    std::vector<int32_t> cls;
    int rc = align_classes(c, pcm, n, std::vector<int32_t>(text_ids, text_ids + n_text), cls, t);
    if (rc) return rc;
    *n_ts = (int)cls.size();
    if (classes) for (int i = 0; i < (int)cls.size() && i < cap; i++) classes[i] = cls[i];
    return 0;
}

// ForcedAligner::tokenize_with_timestamps (src/forced_aligner.cpp:1564-1609)
static std::vector<int32_t> align_tokens(const qasr_model *m, const std::string &text, const std::string &lang,
                                         std::vector<std::string> &words) {
    words = (lang == "korean" && !m->ko_dict.empty()) ? tokenize_korean(text, m->ko_dict) : split_words(text);
    std::vector<int32_t> ids;
    for (const std::string &w : words) {
        std::vector<int32_t> t = m->tok.encode_word(w);
        ids.insert(ids.end(), t.begin(), t.end());
        ids.push_back(m->hp.timestamp_id);
        ids.push_back(m->hp.timestamp_id);
    }
    return ids;
}

extern "C" int qasr_align_tokenize(const qasr_model *m, const char *text, const char *language, int32_t *ids, int cap,
                                   int *n_words) {
    if (!m || !text) return fail(QASR_ERR_ARG, "bad arguments");
    std::vector<std::string> words;
    std::vector<int32_t> v = align_tokens(m, text, language ? language : "", words);
    if (ids) for (int i = 0; i < (int)v.size() && i < cap; i++) ids[i] = v[i];
    if (n_words) *n_words = (int)words.size();
    return (int)v.size();
}

extern "C" int qasr_align_words(const qasr_model *m, const char *text, const char *language, char *out, int cap) {
    if (!m || !text) return -fail(QASR_ERR_ARG, "bad arguments");
    std::vector<std::string> words;
    align_tokens(m, text, language ? language : "", words);
    std::string j;
    for (size_t i = 0; i < words.size(); i++) { if (i) j += '\n'; j += words[i]; }
    if (out && cap > 0) {
        const size_t k = std::min(j.size(), (size_t)cap - 1);
        memcpy(out, j.data(), k);
        out[k] = 0;
    }
    return (int)j.size();
}

extern "C" int qasr_model_load_korean_dict(qasr_model *m, const char *path) {
    if (!m || !path) return fail(QASR_ERR_ARG, "bad arguments");
    if (!load_korean_dict(path, m->ko_dict)) return fail(QASR_ERR_IO, std::string("cannot read Korean dictionary: ") + path);
    return 0;
}

extern "C" int qasr_fix_timestamps(const int32_t *classes, int n, int32_t *out) {
    if (n < 0 || (n && (!classes || !out))) return fail(QASR_ERR_ARG, "bad arguments");
    std::vector<int32_t> r = fix_timestamp_classes(std::vector<int32_t>(classes, classes + n));
    if (n) memcpy(out, r.data(), (size_t)n * 4);
    return 0;
}

static std::string json_escape(const std::string &s) {   // src/main.cpp:230-254
    std::string r;
    for (char ch : s) {
        switch (ch) {
            case '"': r += "\\\""; break;
            case '\\': r += "\\\\"; break;
            case '\b': r += "\\b"; break;
            case '\f': r += "\\f"; break;
            case '\n': r += "\\n"; break;
            case '\r': r += "\\r"; break;
            case '\t': r += "\\t"; break;
            default:
                if ((unsigned char)ch < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", (unsigned char)ch); r += b; }
                else r += ch;
        }
    }
    return r;
}

// whole alignment -> the CLI's JSON document (src/main.cpp:257-276); returns
// the JSON length (excluding NUL) or minus the error code; writes at most
// cap-1 bytes + NUL
static std::string align_doc(const qasr_model *m, const std::vector<std::string> &words, const std::vector<int32_t> &cls, int n);
static int put_str(const std::string &js, char *out, int cap) {
    if (out && cap > 0) {
        const size_t k = std::min(js.size(), (size_t)cap - 1);
        memcpy(out, js.data(), k);
        out[k] = 0;
    }
    return (int)js.size();
}
extern "C" int qasr_align_json(qasr_ctx *c, const float *pcm, int n, const char *text, const char *language, char *out,
                               int cap, qasr_timings *t) {
    if (!c || !pcm || n <= 0 || !text) return -fail(QASR_ERR_ARG, "bad arguments");
    const qasr_model *m = c->m;
    std::vector<std::string> words;
    const std::vector<int32_t> ids = align_tokens(m, text, language ? language : "", words);
    std::vector<int32_t> cls;
    int rc = align_classes(c, pcm, n, ids, cls, t);
    if (rc) return -rc;
    return put_str(align_doc(m, words, cls, n), out, cap);
}

// B clips in one aligner pass (align_classes' batch form): the documents as
// one JSON array, in input order; returns its length or minus the error code
extern "C" int qasr_align_json_batch(qasr_ctx *c, const float *const *pcm, const int *n, const char *const *text, int B,
                                     const char *language, char *out, int cap, qasr_timings *t) {
    if (!c || !pcm || !n || !text || B <= 0) return -fail(QASR_ERR_ARG, "bad arguments");
    const qasr_model *m = c->m;
    std::vector<std::vector<std::string>> words(B);
    std::vector<std::vector<int32_t>> ids(B), cls;
    for (int b = 0; b < B; b++) {
        if (!pcm[b] || n[b] <= 0 || !text[b]) return -fail(QASR_ERR_ARG, "bad arguments");
        ids[b] = align_tokens(m, text[b], language ? language : "", words[b]);
    }
    int rc = align_classes(c, pcm, n, ids, cls, t);
    if (rc) return -rc;
    std::string js = "[";
    for (int b = 0; b < B; b++) js += (b ? ",\n" : "") + align_doc(m, words[b], cls[b], n[b]);
    return put_str(js + "]", out, cap);
}

// the CLI's document for one clip (src/main.cpp:257-276)
static std::string align_doc(const qasr_model *m, const std::vector<std::string> &words, const std::vector<int32_t> &cls, int n) {
    const std::vector<int32_t> fixed = fix_timestamp_classes(cls);
    const float dur = (float)n / 16000.0f, seg = m->hp.ts_segment_ms / 1000.0f;
    std::vector<float> ts(fixed.size());
    for (size_t i = 0; i < fixed.size(); i++) ts[i] = std::min(fixed[i] * seg, dur);
    std::string js = "{\n  \"words\": [\n";
    for (size_t i = 0; i < words.size(); i++) {
        const float st = 2 * i < ts.size() ? ts[2 * i] : 0.0f, en = 2 * i + 1 < ts.size() ? ts[2 * i + 1] : dur;
        char b[64];
        js += "    {\"word\": \"" + json_escape(words[i]) + "\", ";
        snprintf(b, sizeof b, "\"start\": %.3f, \"end\": %.3f}", st, en);
        js += b;
        if (i + 1 < words.size()) js += ",";
        js += "\n";
    }
    js += "  ]\n}";
    return js;
}

// --------------------------------------------------------- host utilities
extern "C" int qasr_load_wav(const char *path, float *out, int max_n, int *sample_rate) {
    std::vector<float> s;
    int sr = 0;
    std::string err;
    if (!path || !load_wav(path, s, sr, err)) { g_err = err.empty() ? "bad path" : err; return -1; }
    if (sample_rate) *sample_rate = sr;
    if (out) memcpy(out, s.data(), (size_t)std::min<int>((int)s.size(), max_n) * 4);
    return (int)s.size();
}

extern "C" int qasr_write_wav(const char *path, const float *pcm, int n, int sample_rate) {
    if (!path || (!pcm && n > 0) || !write_wav(path, pcm, n, sample_rate)) return fail(QASR_ERR_IO, "cannot write wav");
    return 0;
}

extern "C" int qasr_synth_pcm(uint64_t seed, int n, float *out) {
    if (!out || n < 0) return fail(QASR_ERR_ARG, "bad arguments");
    synth_pcm(seed, n, out);
    return 0;
}

// bump with every change to host_util.cpp write_synthetic_gguf's output
extern "C" int qasr_synthetic_gguf_version(void) { return 5; }

extern "C" int qasr_write_synthetic_gguf(const char *path, const char *config, uint64_t seed, int wtype) {
    std::string err;
    if (!path || !config) return fail(QASR_ERR_ARG, "bad arguments");
    if (!write_synthetic_gguf(path, config, seed, wtype, err)) return fail(QASR_ERR_IO, err);
    return 0;
}
