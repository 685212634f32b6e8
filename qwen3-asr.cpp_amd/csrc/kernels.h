// kernels.h -- launch interface of the gfx950 kernels (host-callable).
// All pointers are device pointers; all launches go on the given stream and
// are graph-capturable (no allocation, no synchronisation).
#pragma once

#include <string>

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qasr {

// ---------------------------------------------------------------- mel
struct MelClip {
    long pcm_off;   // first sample of the clip in the packed PCM buffer
    int n;          // samples
    int TF;         // computed frames = n/160 + 1 (last one dropped, src/mel_spectrogram.cpp:517-522)
    long tmp_off;   // offset of [128][TF] fp64 scratch
    long out_off;   // offset of [128][TF-1] fp32 output
};
void launch_mel(const float *pcm, const MelClip *clips, int n_clips, const int2 *blocks, int n_blocks,
                const double2 *tw, const double *hann, const float *filt, double *tmp, unsigned long long *cmax,
                float *out, hipStream_t s);
int mel_frames_per_block();

// ---------------------------------------------------------------- conv front-end
// One entry per 100-frame mel chunk (src/audio_encoder.cpp:331-409).
// conv2 / conv3 weight row length: 9 * channels rounded up to 128, zeros past 9 * channels
inline constexpr int conv_kpad(int channels) { return (9 * channels + 127) / 128 * 128; }

struct ChunkDesc {
    long mel_off;   // element offset of mel[clip][0][chunk_start]
    int T;          // mel row stride (frames of the clip)
    int L;          // chunk frames: ASR = the chunk's own length (last one short, not padded);
                    // aligner = 100 always, zero-padded (src/forced_aligner.cpp:633-698)
    int Lv;         // mel frames read (frames past Lv are zeros); ASR: Lv = L
    int W1, W2, W3; // conv output widths
    int row1, row2, row3;   // first row of this chunk in the conv1/2/3 output tables
    int enc_row;    // first encoder frame (= row3 / 16)
};

// conv1 (1 -> C, 3x3, s2, p1) + bias + GELU(LUT) -> act1 NHWC fp16 [rows1][C]
void launch_conv1(const float *mel, const ChunkDesc *chunks, const int *row1_start, int n_chunks, int rows1,
                  const uint16_t *w /*[C][9]*/, const float *b, const uint16_t *gelu, int C, uint16_t *act1, hipStream_t s,
                  int max_w1 = 50 /* the widest chunk's W1 */);

// ---------------------------------------------------------------- GEMM
enum GemmEpi {
    EPI_F32 = 0,        // out_f32 = acc (+bias) (+res) (+pe[pe_pos[row]])
    EPI_GELU_F16 = 1,   // out_f16 = gelu(acc + bias)
    EPI_SWIGLU_F16 = 2, // interleaved gate/up rows -> out_f16 = silu(g) * u
    EPI_ARGMAX = 3,     // optional out_f32 logits + per-row packed argmax (atomicMax)
    EPI_F16 = 4,        // out_f16 = acc (+bias)
    EPI_SWIGLU_F32 = 5, // as EPI_SWIGLU_F16 with fp32 out_f32 (input of a Q8_0 layer)
    EPI_SWIGLU_Q8 = 6,  // as EPI_SWIGLU_F32, quantised to Q8_0 in the epilogue: out_q / out_d
                        // (the bits of EPI_SWIGLU_F32 + launch_quantize_q8); skinny Q8_0 GEMM only
};
enum GemmAMode {
    AM_DENSE = 0,       // A [M][lda] fp16 row-major
    AM_CONV2 = 1,       // implicit im2col of act1 (NHWC, H=64), rows ordered (chunk, oh, ow)
    AM_CONV3 = 2,       // implicit im2col of act2 (NHWC, H=32), rows ordered (chunk, ow, oh)
};
struct GemmArgs {
    const uint16_t *A; int lda;
    const uint16_t *W; int ldw;     // [N][K] fp16 (PyTorch [out][in])
    int M, N, K;
    // conv gather
    const ChunkDesc *chunks; const int *row_start; int n_chunks; int C;
    // epilogue
    const float *bias;
    const float *res; int ldr;
    float *out_f32; int ldo;
    uint16_t *out_f16; int ldo16;
    const uint16_t *gelu;
    const float *pe; const int *pe_pos;   // conv_out: + PE[pos][n]
    unsigned long long *amax;             // [M] packed argmax keys
    int n_valid;                          // EPI_ARGMAX: columns >= n_valid (zero-padded weight rows) never win; 0 = N
    // Q8_0 operands (launch_gemm_q8): A int8 [M][lda] with fp32 block scales
    // Ad [M][ldad] (one per 32 values), W int8 [N][ldw] with fp16 scales
    // Wd [N][K/32] (ggml block_q8_0 split into quants and scales)
    const int8_t *Aq; const float *Ad; int ldad;
    const int8_t *Wq; const uint16_t *Wd;
    int regs_staged;                      // 1: register-staged tiles instead of the LDS-DMA ones (A/B option)
    int no_skinny;                        // 1: launch_gemm_skinny / _q8 decline (per-context option skinny = 0)
    int skinny_inflight;                  // skinny GEMMs: every K chunk of a wave requested at entry (FuseCfg::skinny_inf)
    int8_t *out_q; float *out_d; int ldoq;   // EPI_SWIGLU_Q8: int8 [M][ldoq], fp32 block scales [M][ldoq / 32]
    int wdef;                             // skinny GEMMs: weights with the default cache policy (1) or nontemporal (0)
};
void launch_gemm(int amode, int epi, const GemmArgs &g, hipStream_t s);
// an unsupported (mode, epilogue) pair launches nothing and is recorded for the
// calling host thread; take_declined returns (and clears) it -- the engine
// fails the call with it (QASR_ERR_STATE) instead of running short
void note_declined(const char *what, int mode, int epi);
bool take_declined(std::string *msg);
// decode-batch GEMM (gemm_skinny.hip): dense A, M <= 128, K % 128 == 0; returns
// false (nothing launched) for shapes it does not take, or when g.no_skinny.
bool launch_gemm_skinny(int epi, const GemmArgs &g, hipStream_t s);
// the same for Q8_0 weights (Aq/Ad quantised activations, Wq/Wd): EPI_F32, EPI_SWIGLU_F32, EPI_SWIGLU_Q8
bool launch_gemm_skinny_q8(int epi, const GemmArgs &g, hipStream_t s);
// ggml_mul_mat with Q8_0 weights: exact int8 block dots (v_mfma_i32_16x16x32_i8
// per 32-wide K block), each scaled by d_w * d_x into an fp32 accumulator.
// Requires K % 128 == 0 (every Qwen3-ASR width) or K % 32 == 0 (slower tile).
void launch_gemm_q8(int epi, const GemmArgs &g, hipStream_t s);
// ggml quantize_row_q8_0 of fp32 (x32) or fp16 (x16) rows [M][K] (row stride
// ldx elements) -> q int8 [M][K], d fp32 [M][K/32] (the fp16-rounded scale).
// gather_C > 0: row element j = c*16 + h is read from column h*gather_C + c
// (the conv_out feature order of src/audio_encoder.cpp:133-142 over the
// [h][c] conv3 activations).
void launch_quantize_q8(const float *x32, const uint16_t *x16, int ldx, int M, int K, int gather_C, int8_t *q, float *d,
                        hipStream_t s);

// skinny (decode) path: M <= 8 rows, weights streamed once from HBM.
// x is fp32 [M][K]; if norm_w != nullptr the rows are RMS-normalised first
// (ggml_rms_norm + ggml_mul), then rounded to fp16 as ggml's mul_mat does.
struct GemvArgs {
    const float *x; int ldx;
    const uint16_t *xh; int ldxh;        // alternative fp16 input (no norm)
    const float *norm_w; float eps;
    const uint16_t *W; int K, N, M;      // N = output columns (for SWIGLU: F outputs)
    const uint16_t *Wd;                  // non-null: W is Q8_0 int8 [N][K] with fp16 scales Wd [N][K/32];
                                         // x (fp32) is quantised per 32 in the prologue (ggml vec_dot_type Q8_0)
    const float *bias;
    const float *res; int ldr;
    float *out_f32; int ldo;
    uint16_t *out_f16; int ldo16;
    unsigned long long *amax;
    // fused embedding gather (decode layer 0): x[m] = embd[ids[m]] (fp16 -> fp32),
    // block 0 also stores it to x_store for the residual stream
    const int32_t *embd_ids; const uint16_t *embd; float *x_store;
    // fused greedy-step bookkeeping (EPI_ARGMAX): the last workgroup decodes the
    // argmax keys into tok_out / hist[b][step+1], advances pos[b] and step,
    // and re-arms amax and done (both zero at rest)
    unsigned int *done; int32_t *tok_out; int32_t *hist; int hist_stride; int *step; int *pos;
    unsigned long long *trace;           // dev trace: per block [start, end, ...] (8 slots, 100 MHz clock) or null
    unsigned int *zero8;                 // gemv1: block 0 re-arms these 8 replicated counters (16-word stride)
    unsigned long long *stamp;           // kernel-duration probe record (dev_common.h stamp_start/end) or null
    int *nkv;                            // launch_lmhead_batch: n_kv[b] += 1 with pos[b] (decode batches) or null
    int n_valid;                         // launch_lmhead_batch: columns >= n_valid never win; 0 = N
    int keep_step;                       // lmhead_batch_kernel: leave *step as it is (a first row-half launch)
};
void launch_gemv(int epi, const GemvArgs &g, hipStream_t s);
// lmhead.hip: decode-batch LM head in one launch (9..128 rows; K = 1024, f16 W):
// RMS norm of x with norm_w, GEMM against W [N][K], optional fp32 logits,
// per-row first-index argmax, and the fused bookkeeping of EPI_ARGMAX above
// (plus nkv); amax and done zero at rest.  false = shape not covered
bool launch_lmhead_batch(const GemvArgs &g, hipStream_t s);
// gemv.hip: one-row f16 fast path of launch_gemv (false = not covered)
bool launch_gemv1(int epi, const GemvArgs &g, hipStream_t s);

// Batch-1 fused launches (a role waits in-launch on another role's output):
// per-context switches, delays and the device's co-residency capacity.  Every
// wait is bounded by poll_limit polls; a wait that runs out sets a bit in the
// sticky device word *err (the host turns it into QASR_ERR_DEVICE) and its
// workgroup skips the dependent store.
enum DevErr : unsigned {
    DEVERR_QKV_WAIT = 1u,    // attention split gave up on its kv group's QKV blocks
    DEVERR_O_WAIT = 2u,      // fused o-projection gave up on the attention combiners
    DEVERR_FFN_WAIT = 4u,    // fused down-projection gave up on the gate/up blocks
    DEVERR_SCORE_WAIT = 8u,  // fused exact attention: the chain gave up on the splits' score granules
};
struct FuseCfg {
    int ffn = 1, qkv = 1, o = 1;        // fused launches on/off
    int ffn_delay = 4, ffn_wdelay = 16; // down blocks: first poll / weight request, s_sleep(8) units (~0.2 us)
    int qkv_delay = 10, o_delay = 32;   // attention K/V request / o-proj weight request delays (o_delay re-swept in
                                        // round 2, tools/experiments.sh delays: 20 -> 26, configs[1] decode 218.4 -> 212.4 ms;
                                        // round 4 with the fp16-V chain, tools/r4/sweep.sh on one box: ffn_wdelay 14 -> 16-18,
                                        // o_delay 26 -> 30-38, 64-key splits to 1.9k keys: 248 -> 263 RTFx)
    int spl1 = 0;                       // batch-1 attention split: 0 = auto (64, or 128 from 1k keys)
    int poll_limit = 1 << 20;           // bounded waits: polls (s_sleep(4..8) apart) before giving up
    int fence = 0;                      // 1 = agent release before each arrival, acquire after each wait
    int enc_attn_f32 = 0;               // encoder attention on fp32 MFMA instead of split fp16 operands
    int gemm_regs = 0;                  // encoder/prefill GEMMs on the register-staged tiles (gemm.hip)
    int gran = 1;                       // batch 1: QKV -> attention hand-off by tagged granules (0 = arrival counters)
    int fa_exact_prefill = 1;           // prefill attention with ggml's CPU FA numerics (fa_exact.hip)
    int fa_exact_decode = 1;            // decode attention likewise: 1 on (every model and batch; batch 1 f16 in the
                                        // fused launch's chain role), 0 off (fp32 V accumulation, split-K)
    int fx_vpf = 2;                     // batch-1 fused exact attention: V^T pulled into L2 ahead of the chain
                                        // (DecodeAttnArgs.fx_vpf bits)
    int slots_ffn = 0, slots_qkv64 = 0, slots_qkv128 = 0;   // co-resident workgroups on this device
    int att_stream = 1;                 // decode batches: one workgroup per (kv group, sequence) (decode_attn_seq_kernel)
    int skinny = 1;                     // decode batches: the weight-streaming skinny GEMMs (0 = tiled GEMMs)
    int att_spl = 256;                  // decode batches on the split attention kernels: keys per split (128 or 256)
    int kv_nt = 1;                      // decode attention: K/V cache rows loaded nontemporal (read once per step by one
                                        // CU; tools/experiments.sh kvnt: configs[1] neutral, 64 x 30 s decode 205.0 -> 202.1 ms)
    int slots_stream = 0;               // ... its co-resident workgroups on this device
    int fx_seq = 1;                     // decode batches: the exact attention's scores + chain in one launch
                                        // (decode_attn_seq_kernel<1>) where the per-sequence kernel is taken
    int lmh = 1;                        // decode batches of f16 models (9..64 rows): the LM head in one launch (lmhead.hip)
    int skinny_inf = 1;                 // decode-batch skinny GEMMs: all of a wave's K chunks in flight (gemm_skinny.hip CPW)
    int skinny_wdef = 1;                // decode-batch skinny GEMMs: weights with the default cache policy (1) or
                                        // nontemporal loads (0) (GemmArgs::wdef; round 6: the row blocks of a column
                                        // tile re-read it from L2 instead of HBM -- utterance set +3.5 %)
    int refill_group = 0;               // qasr_run_stream: at most this many clips a refill (0 = every free slot), so a
                                        // context's refills alternate with its decode steps (small shares)
    int live_prefix = 0;                // qasr_run_stream: decode steps over the slots up to the last live one (16-row
                                        // granules) instead of every slot
    int staged_wrap = 0;                // qasr_run_stream_staged: ids past the staged pool reuse clip id % pool (bench
                                        // utterance sets over a smaller pool); 0: such an id is rejected as out of range
    int poison = 0;                     // test only: scratch buffers grown by the context are filled with 0xFF bytes
                                        // (fp16 NaN) so a kernel reading rows it never wrote shows up in its outputs
    unsigned int *err = nullptr;        // sticky device error word (DevErr bits)
};
// co-resident workgroup capacity of the fused kernels on the current device
// (occupancy query x CUs); 0 = unknown (never fuse)
void fused_slots(FuseCfg &cfg);
// hand-off state of the batch-1 FFN roles (ffn_roles.h)
struct FfnCtl {
    unsigned int *cnt, *cnt_next;   // this layer's 32 gate/up arrival shards (16-word stride), the next layer's
    unsigned int *err;              // sticky device error word
    int wdelay, delay, poll_limit, fence;
};
// gemv.hip: batch-1 f16 gate/up + down in one launch; cnt = this layer's
// 32 x 16 words (zero on entry), cnt_next = the next layer's, re-armed here
// (false = not covered; dry: the decision only)
bool launch_ffn1(const GemvArgs &gu, const GemvArgs &dn, unsigned int *cnt, unsigned int *cnt_next, const FuseCfg &cfg,
                 hipStream_t s, bool dry = false);

// ---------------------------------------------------------------- norms
// LayerNorm (ggml_norm + mul + add) fp32 [M][D] -> fp16 y, or fp32 y32 when
// non-null (input of a Q8_0 layer)
void launch_layernorm_f16(const float *x, int M, int D, const float *w, const float *b, float eps, uint16_t *y, hipStream_t s,
                          float *y32 = nullptr);
// RMSNorm (ggml_rms_norm + mul) fp32 -> fp16 (or fp32 y32); rows gathered by optional row_idx
void launch_rmsnorm_f16(const float *x, int ldx, const int *row_idx, int M, int D, const float *w, float eps,
                        uint16_t *y, hipStream_t s, float *y32 = nullptr);
// the same norm quantised to Q8_0 in the kernel (decode batches of Q8_0 models):
// yq int8 [M][D], yd fp32 [M][D/32] -- the values launch_quantize_q8 would give
void launch_rmsnorm_q8(const float *x, int ldx, int M, int D, const float *w, float eps, int8_t *yq, float *yd, hipStream_t s);

// ---------------------------------------------------------------- attention
// encoder: full bidirectional attention per clip segment, head_dim 64, fp32-level
// arithmetic (split fp16 operands on f16 MFMA, or fp32 MFMA when f32_mfma).
// qkv fp32 [rows][3*D]; out fp16 [rows][D] (or fp32 out32 when non-null)
void launch_enc_attention(const float *qkv, const int *seg_start, const int *seg_len, int n_seg, int max_len,
                          int D, int H, uint16_t *out, hipStream_t s, float *out32 = nullptr, bool f32_mfma = false);

// rows of padding after the last K/V cache region: the exact-attention chains
// (fa_exact.hip) load V a few batches ahead without clamping
constexpr long kKvPadRows = 256;
// V^T cache for the decode chain of fa_exact.hip: per (layer, slot, kv head)
// vt_ctx / 8 key blocks of [128 d][8 keys] fp16 -- one dimension's 8 keys in
// 16 B, a wave's 64 dimensions of a block in 1 KiB contiguous (a plain
// [d][key] layout put every lane of a load on its own page).  vt_ctx =
// max_ctx rounded up to 64 plus 384 keys of read-ahead slack.
__host__ __device__ inline int vt_ctx(int max_ctx) { return (max_ctx + 63) / 64 * 64 + 384; }
// element (key k, dimension d) of one (slot, kv head) region
__host__ __device__ inline long vt_index(int k, int d) { return ((long)(k >> 3) * 128 + d) * 8 + (k & 7); }

// decoder q/k RMSNorm + NEOX RoPE + fp16 KV-cache write (+ q fp16 out)
struct QkvPostArgs {
    const float *qkv; int rows;          // [rows][QD + 2*KD] fp32 from the fused QKV GEMM
    const int *row_seq; const int *row_pos;   // per row: sequence slot, absolute position
    const float *q_norm, *k_norm; float eps;
    const float *rope;                   // [max_pos][64][2]
    int n_head, n_kv_head;               // head_dim fixed at 128
    uint16_t *q_out;                     // [rows][n_head*128] fp16
    uint16_t *kc, *vc;                   // this layer's cache base: [seq][kvh][max_ctx][128]
    int max_ctx;
    uint16_t *vt;                        // this layer's V^T cache base: [seq][kvh][128][vt_ctx(max_ctx)]
    float *q32, *k32;                    // non-null (ForcedAligner): also the fp32 rows [rows][QD] / [rows][KD]
};
void launch_qkv_post(const QkvPostArgs &a, hipStream_t s);

// decoder causal prefill attention (fp16 Q/K/V, fp32 softmax), GQA 2:1, hd 128
struct PrefillAttnArgs {
    const uint16_t *q;                   // [rows][n_head*128]
    const uint16_t *kc, *vc;             // layer cache base
    const int *seq_row0; const int *seq_len; const int *seq_slot; int n_seq; int max_len;
    int n_head, n_kv_head, max_ctx;
    float scale;
    uint16_t *out;                       // [rows][n_head*128] fp16
    float *out32;                        // non-null: fp32 output instead (input of a Q8_0 o-proj)
    int8_t *outq; float *outd;           // non-null: Q8_0 output [B][QD] int8 + [B][QD/32] scales
    const float *q32, *k32;              // non-null (exact kernel only): fp32 scores from these fp32 rows, key k of
                                         // sequence s at row seq_row0[s] + k (the aligner's K stays fp32,
                                         // src/forced_aligner.cpp:1041-1046)
    const int *seq_pos0;                 // non-null: sequence s's rows sit at positions seq_pos0[s] + t (a chunk after
                                         // seq_pos0[s] cached tokens, TextDecoder::forward at n_past > 0); keys
                                         // 0 .. seq_pos0[s] + seq_len[s] - 1, causal by position (not with q32/k32)
};
void launch_prefill_attention(const PrefillAttnArgs &a, hipStream_t s);
// the same attention with ggml's CPU flash-attention numerics (fa_exact.hip):
// keys in order per query row, fp16 V accumulator rounded after every key
void launch_prefill_attention_exact(const PrefillAttnArgs &a, hipStream_t s);
// fa_exact.hip: the exact prefill kernel's expf (px_expf_nonpos) against the
// device expf on all 2^31 non-positive inputs, on the current device
hipError_t check_expf_nonpos(unsigned long long *mismatches);

// row stride (granules) of the fused exact attention's score granules
__host__ __device__ inline int sgran_ld(int max_ctx) { return (max_ctx + 63) / 64 * 64; }
// tag of a batch-1 hand-off granule {value, tag} (DecodeAttnArgs.gran): the
// step's position and the layer.  Never 0, the value the granule buffers are
// reset to before every call, so a granule not yet written this step can
// never match (position 0 at layer 0 included).
__host__ __device__ inline uint32_t gran_tag(int pos, int layer) { return ((uint32_t)(pos + 1) << 5) | (uint32_t)layer; }

// decoder single-token attention, fused: q/k RMSNorm + RoPE, fp16 KV-cache
// write of the new token and split-KV flash decoding (64-key splits); the last
// arriving split of each kv group combines the partials and writes out.
struct DecodeAttnArgs {
    const float *qkv;                    // [B][QD + 2*KD] fp32 (raw QKV projection)
    const float *q_norm, *k_norm; float eps;
    const float *rope;                   // [max_pos][64][2]
    const int *pos;                      // [B] position of the fed token (n_past)
    uint16_t *kc, *vc;                   // this layer's cache base
    uint16_t *vt;                        // this layer's V^T cache base (the new token's V is written there too)
    const int *seq_slot;
    int B, n_head, n_kv_head, max_ctx, max_splits;
    int grid_splits;                     // launched splits: >= ceil((max pos + 1) / 64) over the batch
    float scale;
    float *part;                         // [B][n_kv_head][max_splits][2][132]: O[128], m, l, 0, 0
    unsigned int *counter;               // [B][n_kv_head] split arrivals, zero at rest
    uint16_t *out;                       // [B][n_head*128] fp16 attention output
    float *out32;                        // non-null: fp32 output instead (input of a Q8_0 o-proj)
    int8_t *outq; float *outd;           // non-null: Q8_0 output [B][QD] int8 + [B][QD/32] scales
    unsigned long long *trace;           // dev trace: per block [start, K/V landed, partial ready, counted, end, burst landed]
    unsigned int *qcnt;                  // [n_kv_head][8 replicas][16] QKV-block arrivals of the fused batch-1 launch, zero at rest
    int fuse_delay;                      // fused launch: attention blocks idle fuse_delay x ~0.2 us before their K/V loads
    unsigned int *att_done;              // [8 replicas][16] combiner arrivals for the fused o-proj (re-armed by the down-proj)
    int oproj_delay;                     // fused launch: o-proj blocks idle oproj_delay x ~0.2 us before their weight loads
    int poll_limit;                      // fused launch: bounded waits (FuseCfg)
    int fence;                           // fused launch: agent release/acquire around the hand-offs (FuseCfg)
    unsigned int *err;                   // fused launch: sticky device error word (DevErr bits)
    int spl1;                            // batch <= 8: key split (0 = auto: 64, or 128 from 1k keys)
    unsigned long long *stamp;           // kernel-duration probe record or null
    unsigned int qkv_need;               // fused launches: QKV-block arrivals per kv group (0 = 64)
    float *scores;                       // non-null (separate launch only): scores mode -- the splits write their
                                         // scaled scores [B][n_head][max_ctx] (+ the new K/V rows) and stop there
    unsigned long long *gran;            // fused launch: QKV outputs as 8-byte {fp32 value, tag} granules the attention
                                         // splits poll directly (no drain / arrival count); null = counters
    int layer;                           // granule tag = gran_tag(position, layer)
    int stream_blocks;                   // decode batches (B > 8): co-resident workgroups of decode_attn_seq_kernel (one per
                                         // kv group and sequence, taken once the batch fills them; 0 = split kernels)
    int spl_batch;                       // decode batches on the split kernels: 128- or 256-key splits (FuseCfg::att_spl)
    int kv_nt;                           // K/V cache loads nontemporal (FuseCfg::kv_nt)
    int fx_seq;                          // decode batches on the per-sequence kernel: exact attention in one launch (FuseCfg::fx_seq)
    // batch-1 fused launch with ggml's fp16-accumulating attention (fx = 1,
    // needs gran): the splits publish their scaled scores as {fp32, tag}
    // granules in sgran [n_head][max_ctx]; one chain workgroup per kv group
    // runs fx_chain.h's chain for both query heads and hands the output to the
    // o-projection role (att_done)
    int fx;
    unsigned long long *sgran;           // row stride sgran_ld(max_ctx) (16-B aligned granule pairs)
    int fx_vpf;                          // bit 0: the splits pull their keys' V^T rows into their XCD's L2 for the
                                         // chain; bit 1: the chain workgroups pull their own (LDS-DMA, while waiting)
};
// the decode attention with ggml's CPU flash-attention numerics (fa_exact.hip),
// after launch_decode_attention in scores mode: per (query head, sequence) the
// keys in order with the fp16 V accumulator; reads scores, pos, vc, n_head,
// n_kv_head, max_ctx and writes one of out / out32 / outq+outd
void launch_decode_attention_exact(const DecodeAttnArgs &a, hipStream_t s);
// attention.hip: scores + that chain in one launch for decode batches on the
// per-sequence kernel (a.fx_seq); false = not covered, run the two launches
bool launch_decode_attention_exact_seq(const DecodeAttnArgs &a, hipStream_t s);

void launch_decode_attention(const DecodeAttnArgs &a, hipStream_t s);
// batch 1, f16: the QKV projection (q: GemvArgs of the rmsnorm+QKV GEMV, K = 1024)
// and the attention in one launch (attention.hip); false = not taken
// (and, when o is the plain batch-1 o-projection, that too); returns 0 = not
// taken, 1 = QKV + attention, 2 = QKV + attention + o-projection
// dry = true: only the decision (nothing launched)
int launch_qkv_attention1(const GemvArgs &q, const DecodeAttnArgs &a, const GemvArgs *o, const FuseCfg &cfg, hipStream_t s,
                          bool dry = false);
int decode_split_len();
int decode_max_splits();

// ---------------------------------------------------------------- decoder misc
// embedding gather (fp16 -> fp32) + audio splice (src/text_decoder.cpp:429-459)
void launch_embed(const int32_t *ids, int rows, const uint16_t *embd, int hidden, const float *audio,
                  const int *row_audio /* -1 or audio row */, float *x, hipStream_t s);
// final argmax decode of packed keys -> ids; optionally scatter into a token history
void launch_argmax_finish(const unsigned long long *amax, int B, int32_t *ids, int32_t *hist, int hist_stride,
                          const int *step, hipStream_t s);
void launch_fill_u64(unsigned long long *p, int n, unsigned long long v, hipStream_t s);
// dst row r = src row idx[r], fp32 rows of D floats (D % 4 == 0)
void launch_gather_rows(const float *src, const int *idx, int rows, int D, float *dst, hipStream_t s);
// decode-step bookkeeping on device: n_kv[b] += 1, row_pos[b] += 1, step += 1
void launch_step_advance(int *row_pos, int *n_kv, int *step, int B, hipStream_t s);

}  // namespace qasr
