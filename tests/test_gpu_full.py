"""GPU parity at the real Qwen3-ASR-0.6B dimensions (synthetic f16 weights,
reference tensor names/shapes: 18 x 896 encoder, 28 x 1024 decoder,
151936 vocab).  Sizes are kept where the CPU oracle finishes in seconds;
the full 30 s / 92 s workloads are covered by size-independent properties
(batch == single, determinism, decode budget) and by bench.py."""
import os

import numpy as np
import pytest

import oracle_py as op
import qasr

pytestmark = pytest.mark.gpu
SR = 16000


# Absolute bars beside the relative ones, set from the recorded measurements
# (profiles/r4/parity.json) with ~2x margin: the reference's own decoder bar is
# absolute 1e-2 (tests/test_decoder.cpp:157) at a real model's logit scale;
# the synthetic weights give a logit scale of ~18, where the measured max
# |delta| is 0.017-0.027 (about 1.2e-3 of the scale).
ABS_LOGITS = 5e-2
REL_LOGITS = 3e-3


def _err(g, o):
    """(absolute max |delta|, that / max |oracle|): the reference's own decoder
    bar is absolute 1e-2 (tests/test_decoder.cpp:157); with random-init weights
    the logit scale is ~20x a real model's spread.  The tests hold both the
    relative 1e-2 of before and the measured-plus-margin bars above."""
    d = float(np.abs(np.asarray(g, np.float64) - np.asarray(o, np.float64)).max())
    return d, d / float(np.abs(o).max())


@pytest.fixture(scope="module")
def full(gpu, full_f16_gguf):
    p = full_f16_gguf
    m = qasr.Model(p)
    c = qasr.Context(m, max_batch=4, max_ctx=1536)
    op.set_threads(min(16, os.cpu_count() or 1))
    om = op.OracleModel(p)
    yield m, c, om
    c.close()
    m.close()


def test_full_hparams(full):
    m, _, _ = full
    hp = m.hp
    assert (hp.enc_layers, hp.d_model, hp.enc_heads, hp.enc_ffn, hp.conv_channels) == (18, 896, 14, 3584, 480)
    assert (hp.vocab_size, hp.hidden_size, hp.dec_layers, hp.n_heads, hp.n_kv_heads, hp.head_dim, hp.dec_ffn) == (
        151936, 1024, 28, 16, 8, 128, 3072)
    assert m.device_bytes > 1.5e9


@pytest.mark.parametrize("secs", [1.0, 3.1])
def test_full_encode(full, secs):
    _, c, om = full
    mel = op.log_mel(qasr.synth_pcm(11000, int(secs * SR)))
    g = c.encode([mel])[0]
    o = om.encode(mel)
    d = np.abs(g - o)
    assert g.shape == o.shape == (qasr.encoder_frames(mel.shape[1]), 1024)
    assert d.max() <= 2e-2 and d.mean() <= 1e-3, (d.max(), d.mean())


def test_full_prefill_and_steps(full, parity):
    m, c, om = full
    mel = op.log_mel(qasr.synth_pcm(12000, 2 * SR))
    feats = om.encode(mel)
    ids, pos = m.build_prompt(feats.shape[0])
    lg, am = c.prefill([ids], [feats], [pos])
    d = op.OracleDecoder(om, 256)
    lo = d.forward(ids, 0, feats, pos)
    ab, rel = _err(lg[0], lo)
    errs = [(ab, rel)]
    assert rel <= REL_LOGITS and ab <= ABS_LOGITS, (ab, rel)
    rng = np.random.default_rng(3)
    n_past = len(ids)
    for _ in range(6):   # batch 1, f16: the fused launch with ggml's fp16-accumulating attention (the default)
        tok = int(rng.integers(0, 151643))
        lg, am = c.decode_step([tok], [n_past])
        lo = d.forward([tok], n_past)
        ab, rel = _err(lg[0], lo)
        errs.append((ab, rel))
        assert rel <= REL_LOGITS and ab <= ABS_LOGITS, (ab, rel)
        n_past += 1
    parity("full_2s_prefill_and_6_steps", abs_max=[e[0] for e in errs], rel_max=[e[1] for e in errs],
           scale=float(np.abs(lo).max()), fused_exact=c.get_option("fused_exact"))


def test_full_transcribe_tokens(full):
    _, c, om = full
    pcm = qasr.synth_pcm(13000, 2 * SR)
    r = c.transcribe([pcm], max_tokens=8, ignore_eos=True)
    ora, _ = om.transcribe(pcm, max_tokens=8, ignore_eos=True)
    assert r.tokens[0] == ora


def test_full_batch64_rows_identical(full):
    """the bench's batch shapes (64 rows: skinny QKV / o / gate-up / down and
    LM-head tilings of the 0.6B model): 64 identical clips give 64 identical
    token streams, and the first token equals the batch-1 (GEMV) path's"""
    m, c, _ = full
    pcm = qasr.synth_pcm(9300, int(1.1 * SR))
    cb = qasr.Context(m, max_batch=64, max_ctx=128)
    try:
        r = cb.transcribe([pcm] * 64, max_tokens=6, ignore_eos=True)
    finally:
        cb.close()
    r1 = c.transcribe([pcm], max_tokens=6, ignore_eos=True)
    assert all(t == r.tokens[0] for t in r.tokens)
    assert len(r.tokens[0]) == 6 and r.tokens[0][0] == r1.tokens[0][0]


def test_full_30s_batch_properties(full):
    """30 s clips (configs[0]/[2] length): batched == single, deterministic,
    budget met, token ids in range."""
    _, c, _ = full
    clips = [qasr.synth_pcm(14000 + i, 30 * SR) for i in range(2)]
    rb = c.transcribe(clips, max_tokens=24, ignore_eos=True)
    rb2 = c.transcribe(clips, max_tokens=24, ignore_eos=True)
    assert rb.tokens == rb2.tokens
    for pcm, t in zip(clips, rb.tokens):
        assert len(t) == 24 and all(0 <= x < 151936 for x in t)
        assert c.transcribe([pcm], max_tokens=24, ignore_eos=True).tokens[0] == t


def test_full_lds_dma_gemm_bit_identical(full):
    """The LDS-DMA GEMM tiles (the default for >= 2048-row projections and the
    implicit-GEMM convs) multiply the same fragments in the same k order as the
    register-staged tiles (option gemm_regs): encoder features of 8 x 30 s
    clips (3120 rows) and the batch's prefill logits (3240 rows) bit-identical,
    and the batched features equal to a single clip's (small-M tiles)."""
    m, _, _ = full
    clips = [qasr.synth_pcm(15000 + i, 30 * SR) for i in range(8)]
    cb = qasr.Context(m, max_batch=8, max_ctx=512)
    try:
        mels = cb.mel(clips)
        out = {}
        for regs in (1, 0):
            cb.set_option("gemm_regs", regs)
            f = cb.encode(mels)
            ids, pos = m.build_prompt(f[0].shape[0])
            lg, _ = cb.prefill([ids] * 8, f, [pos] * 8)
            out[regs] = (f, lg)
        single = cb.encode([mels[3]])[0]
    finally:
        cb.close()
    for a, b in zip(out[0][0], out[1][0]):
        assert np.array_equal(a, b)
    assert np.array_equal(np.asarray(out[0][1]), np.asarray(out[1][1]))
    assert np.array_equal(single, out[0][0][3])


def test_full_encoder_ragged_tiles_bit_identical(full):
    """Ragged clips (short last chunks, row counts no multiple of 256): the
    8-phase tile's shifted last row / column tiles and its implicit-im2col
    convs against the register-staged tiles (option gemm_regs), bit for bit."""
    m, _, _ = full
    secs = [29.37, 17.71, 8.13, 30.0, 3.05]
    clips = [qasr.synth_pcm(15500 + i, int(s * SR)) for i, s in enumerate(secs)]
    cb = qasr.Context(m, max_batch=len(clips), max_ctx=512)
    try:
        mels = cb.mel(clips)
        out = {}
        for regs in (1, 0):
            cb.set_option("gemm_regs", regs)
            out[regs] = cb.encode(mels)
    finally:
        cb.close()
    for a, b in zip(out[0], out[1]):
        assert a.shape == b.shape and np.array_equal(a, b)


def test_full_encoder_poisoned_scratch(full):
    """the implicit-im2col convs must never read activation rows they
    did not write (the 8-phase tile's K-padding taps read the zero line).  With
    option poison_scratch every scratch buffer the context grows starts as 0xFF
    bytes (fp16 NaN): odd-width chunks (ragged clips, conv3 at W2 = 25) and a
    long odd-length encode_no_chunk clip (conv2 through the 8-phase tile at odd
    W1) give the same finite features as a clean context, bit for bit."""
    m, _, _ = full
    secs = [29.37, 17.71, 30.0]
    clips = [qasr.synth_pcm(15600 + i, int(s * SR)) for i, s in enumerate(secs)]
    long_clip = qasr.synth_pcm(15650, int(47.31 * SR))
    out = {}
    for poison in (0, 1):
        cb = qasr.Context(m, max_batch=len(clips), max_ctx=512)
        try:
            cb.set_option("poison_scratch", poison)
            mels = cb.mel(clips)
            f = cb.encode(mels)
            nc = cb.encode_no_chunk(cb.mel([long_clip]))[0]
            out[poison] = (f, nc)
        finally:
            cb.close()
    for a, b in zip(out[0][0], out[1][0]):
        assert np.isfinite(b).all() and np.array_equal(a, b)
    assert np.isfinite(out[1][1]).all() and np.array_equal(out[0][1], out[1][1])


FUSE_KNOBS = {"QASR_FUSE_FFN": dict(fuse_ffn=0), "QASR_FUSE_QKV": dict(fuse_qkv=0, fuse_o=0), "QASR_FUSE_O": dict(fuse_o=0)}


def _step_state(c, ids, feats, pos, tok=1234):
    """prefill + one decode step: logits and the decode-state buffers"""
    c.prefill([ids], [feats], [pos])
    lg, _ = c.decode_step([tok], [len(ids)])
    return lg[0].copy(), {k: c.debug_read(k)[0].copy() for k in ("x", "act", "qkv", "att")}


@pytest.mark.parametrize("exact", [1, 0])
@pytest.mark.parametrize("knob", list(FUSE_KNOBS))
def test_full_fused_launches_match_separate(full, knob, exact):
    """A batch-1 fused launch (gate/up + down; QKV + attention (+ o-proj))
    against the separate launches of the same arithmetic, switched per context
    (qasr_ctx_set_option): bit-identical decode-step logits and state, and the
    same greedy tokens.  exact = 1 (the default): the fused launch's chain role
    (ggml's fp16 V accumulation) against the separate scores + chain kernels of
    fa_exact.hip; exact = 0: the fp32-accumulating split-K attention (option).
    (Round 1 saw up to 0.0098 here: LLVM folded fp16(fp32 product) into
    v_fma_mixlo_f16 in one kernel and not the other -- dev_common.h rn32.)"""
    m, _, om = full
    c1 = qasr.Context(m, max_batch=1, max_ctx=512)
    c1.set_option("fa_exact_decode", exact)
    try:
        pcm = qasr.synth_pcm(14000, 3 * SR)
        feats = c1.encode(c1.mel([pcm]))[0]
        ids, pos = m.build_prompt(feats.shape[0])
        r_f = c1.transcribe([pcm], max_tokens=24, ignore_eos=True)
        lg_f, st_f = _step_state(c1, ids, feats, pos)
        for k, v in FUSE_KNOBS[knob].items():
            c1.set_option(k, v)
        r_s = c1.transcribe([pcm], max_tokens=24, ignore_eos=True)
        lg_s, st_s = _step_state(c1, ids, feats, pos)
    finally:
        c1.close()
    assert r_f.tokens == r_s.tokens
    assert np.array_equal(lg_f, lg_s), float(np.abs(lg_f - lg_s).max())
    for k in st_f:
        assert np.array_equal(st_f[k], st_s[k]), k
    d = op.OracleDecoder(om, 512, 0 if exact else op.OracleModel.FA_V_F32)
    d.forward(ids, 0, feats, pos)
    lo = d.forward([1234], len(ids))
    ab, rel = _err(lg_f, lo)
    assert rel <= 1e-2, (ab, rel)


def test_full_decode_from_position_zero(full):
    """decode_step at n_past = 0 (no prompt: the first key is the fed token's
    own) through the fused launch -- the granule tags of position 0 / layer 0
    must not match the zeroed buffers -- bit-identical to the separate launches
    and within the bar of the oracle"""
    m, _, om = full
    c1 = qasr.Context(m, max_batch=1, max_ctx=257)   # (odd: the score-granule rows are padded)
    try:
        out = {}
        for fused in (1, 0):
            c1.set_option("fuse_qkv", fused)
            c1.set_option("fuse_o", fused)
            lgs = []
            for k, tok in enumerate([151644, 8948, 198]):
                lg, _ = c1.decode_step([tok], [k])
                lgs.append(lg[0].copy())
                # fused: QKV + attention + o-proj (mode 2)
                assert c1.get_option("fused_exact") == fused and c1.get_option("fused_mode") == 2 * fused
            out[fused] = lgs
    finally:
        c1.close()
    d = op.OracleDecoder(om, 256)
    for k, tok in enumerate([151644, 8948, 198]):
        lo = d.forward([tok], k)
        assert np.array_equal(out[1][k], out[0][k]), (k, float(np.abs(out[1][k] - out[0][k]).max()))
        ab, rel = _err(out[1][k], lo)
        assert rel <= 1e-2, (k, ab, rel)


def test_full_fused_launches_long_context(full):
    """80 s clip (prompt ~1.06k tokens: 128-key attention splits, 10 per kv
    group): fused and separate launches give the same 24 greedy tokens and
    bit-identical decode-step logits."""
    m, _, _ = full
    c1 = qasr.Context(m, max_batch=1, max_ctx=1280)
    try:
        pcm = qasr.synth_pcm(15000, 80 * SR)
        r_f = c1.transcribe([pcm], max_tokens=24, ignore_eos=True)
        feats = c1.encode(c1.mel([pcm]))[0]
        ids, pos = m.build_prompt(feats.shape[0])
        lg_f, _ = _step_state(c1, ids, feats, pos)
        for k in ("fuse_ffn", "fuse_qkv", "fuse_o"):
            c1.set_option(k, 0)
        r_s = c1.transcribe([pcm], max_tokens=24, ignore_eos=True)
        lg_s, _ = _step_state(c1, ids, feats, pos)
    finally:
        c1.close()
    assert r_f.tokens == r_s.tokens
    assert np.array_equal(lg_f, lg_s), float(np.abs(lg_f - lg_s).max())


def test_full_fused_wait_timeout_is_an_error(full):
    """A bounded in-launch wait that runs out is reported (QASR_ERR_DEVICE
    through qasr_last_error), never silently consumed; the context works again
    once the bound is restored."""
    m, _, _ = full
    c1 = qasr.Context(m, max_batch=1, max_ctx=256)
    try:   # every fused launch in play (chain role included)
        # (the QKV launch: 512 QKV blocks, the splits, 8 chain blocks, 256 o-proj blocks)
        assert c1.get_option("slots_ffn") >= 1024 + 256 and c1.get_option("slots_qkv") >= 512 + 8 * 4 + 8 + 256
        pcm = qasr.synth_pcm(14000, 2 * SR)
        ref = c1.transcribe([pcm], max_tokens=4, ignore_eos=True).tokens
        for k, v in (("poll_limit", 1), ("ffn_delay", 0), ("ffn_wdelay", 0), ("qkv_delay", 0), ("o_delay", 0)):
            c1.set_option(k, v)
        with pytest.raises(qasr.QasrError, match="timed out"):
            c1.transcribe([pcm], max_tokens=4, ignore_eos=True)
        c1.set_option("poll_limit", 1 << 20)
        assert c1.transcribe([pcm], max_tokens=4, ignore_eos=True).tokens == ref
    finally:
        c1.close()


def test_full_two_threads_one_device(full):
    """Contexts driven from two host threads on one GPU: the calls that can
    take the fused batch-1 launches hold the device's lock (a fused launch
    needs every CU), so both threads get the same ids as sequential runs and
    no in-launch wait times out."""
    import threading
    m, _, _ = full
    clips = [qasr.synth_pcm(16000 + i, 2 * SR) for i in range(2)]
    ctxs = [qasr.Context(m, max_batch=1, max_ctx=256) for _ in range(2)]
    try:
        ref = [ctxs[i].transcribe([clips[i]], max_tokens=16, ignore_eos=True).tokens[0] for i in range(2)]
        out, err = [None, None], []

        def work(i):
            try:
                for _ in range(3):
                    out[i] = ctxs[i].transcribe([clips[i]], max_tokens=16, ignore_eos=True).tokens[0]
            except Exception as e:   # noqa: BLE001
                err.append(e)
        th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not err, err
        assert out == ref
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.timeout(900)
def test_full_configs1_92s(full, parity):
    """configs[1] at its full size (92 s clip, N = 1196 encoder frames,
    P = 1211 prompt tokens): mel, encoder, prefill logits and 15
    teacher-forced decode steps against the oracle, and the first 16 greedy
    tokens of the whole GPU path exactly the oracle's."""
    _, c, om = full
    pcm = qasr.synth_pcm(16000, 92 * SR)
    mel_o = op.log_mel(pcm)
    mel_g = c.mel([pcm])[0]
    assert mel_g.shape == mel_o.shape == (128, 9200)
    assert np.abs(mel_g - mel_o).max() <= 1e-5
    feats_o = om.encode(mel_o)
    feats_g = c.encode([mel_o])[0]
    assert feats_o.shape == (1196, 1024)
    d = np.abs(feats_g - feats_o)
    parity("configs1_92s_encoder", abs_max=float(d.max()), abs_mean=float(d.mean()), mel_abs_max=float(np.abs(mel_g - mel_o).max()))
    # the reference's bar (max 2e-2, mean 1e-3, tests/run_all_tests.sh:166) and the measured 1.7e-3 / 2.8e-4 with margin
    assert d.max() <= 5e-3 and d.mean() <= 5e-4, (d.max(), d.mean())
    ids, pos = om.prompt(1196), 9
    assert len(ids) == 1211
    dec = op.OracleDecoder(om, 1300)
    lo = [dec.forward(ids, 0, feats_o, pos)]
    toks = [int(np.argmax(lo[0]))]
    for k in range(1, 16):
        lo.append(dec.forward([toks[-1]], len(ids) + k - 1))
        toks.append(int(np.argmax(lo[-1])))
    lg, am = c.prefill([ids], [feats_o], [pos])
    ab, rel = _err(lg[0], lo[0])
    print(f"configs[1] prefill logits: max |d| {ab:.4g} abs, {rel:.3g} of scale")
    assert rel <= 1e-2, (ab, rel)
    assert int(am[0]) == toks[0]
    # 15 teacher-forced decode steps on the oracle's tokens in the default mode:
    # the fused batch-1 launch with ggml's fp16 V accumulation (chain role)
    assert c.get_option("fa_exact_decode") == 1
    c.prefill([ids], [feats_o], [pos])
    errs = []
    for k in range(1, 16):
        lg, am = c.decode_step([toks[k - 1]], [len(ids) + k - 1])
        assert c.get_option("fused_exact") == 1
        errs.append(_err(lg[0], lo[k]))
    print("configs[1] decode steps (abs, rel):", [(round(a_, 4), round(r_, 5)) for a_, r_ in errs])
    r = c.transcribe([pcm], max_tokens=16, ignore_eos=True)
    parity("configs1_92s_prefill_and_15_steps", prefill_abs=ab, prefill_rel=rel, steps_abs=[e[0] for e in errs],
           steps_rel=[e[1] for e in errs], scale=float(np.abs(lo[1]).max()), greedy16_equal=r.tokens[0] == toks)
    assert rel <= REL_LOGITS and ab <= ABS_LOGITS, (ab, rel)
    assert max(r_ for _, r_ in errs) <= REL_LOGITS and max(a_ for a_, _ in errs) <= ABS_LOGITS, errs
    assert r.tokens[0] == toks


@pytest.mark.timeout(900)
def test_full_configs2_q8_b64_30s(gpu, full_q8_gguf, parity):
    """configs[2] at its full size: Qwen3-ASR-0.6B Q8_0 (synthetic weights),
    64 x 30 s clips (P = 405 prompt tokens each, 105-token budget).  All 64
    rows bit-identical (identical clips), every budget met, and row 0 against
    the default-flag oracle: prefill logits and the first decode step within the
    Q8_0 bars of tests/test_gpu_q8.py (1e-2 x the logit scale, or 2.5 x the
    oracle's own sensitivity to a 1e-6 perturbation of the encoder features,
    whichever is larger).  The decode attention runs the exact (fp16 V
    accumulation) kernels, the Q8_0 default."""
    p = full_q8_gguf
    op.set_threads(min(16, os.cpu_count() or 1))
    om = op.OracleModel(p)
    m = qasr.Model(p)
    B, n, budget = 64, 30 * SR, 105
    pcm = qasr.synth_pcm(17000, n)
    mel = op.log_mel(pcm)
    feats = om.encode(mel)
    ids, pos = m.build_prompt(feats.shape[0])
    assert len(ids) == 405
    c = qasr.Context(m, max_batch=B, max_ctx=len(ids) + budget + 8)
    try:
        assert c.get_option("fa_exact_decode") == 1   # the default: exact
        r = c.transcribe([pcm] * B, max_tokens=budget, ignore_eos=True)
        assert all(len(t) == budget for t in r.tokens)
        assert all(t == r.tokens[0] for t in r.tokens)
        lg, am = c.prefill([ids] * B, [feats] * B, [pos] * B)
        for b in range(1, B):
            assert np.array_equal(lg[b], lg[0]), b
        tok0 = int(am[0])
        lg1, _ = c.decode_step([tok0] * B, [len(ids)] * B)
        for b in range(1, B):
            assert np.array_equal(lg1[b], lg1[0]), b
    finally:
        c.close()
        m.close()
    rng = np.random.default_rng(5)
    featsn = (feats * (1 + 1e-6 * rng.standard_normal(feats.shape))).astype(np.float32)
    d, dn = op.OracleDecoder(om, len(ids) + 8), op.OracleDecoder(om, len(ids) + 8)
    lo, ln = d.forward(ids, 0, feats, pos), dn.forward(ids, 0, featsn, pos)
    tol = max(1e-2 * float(np.abs(lo).max()), 2.5 * float(np.abs(lo - ln).max()))
    lo1, ln1 = d.forward([tok0], len(ids)), dn.forward([tok0], len(ids))
    tol1 = max(1e-2 * float(np.abs(lo1).max()), 2.5 * float(np.abs(lo1 - ln1).max()))
    parity("configs2_q8_b64_30s_row0", prefill_abs=float(np.abs(lg[0] - lo).max()), prefill_tol=tol,
           step1_abs=float(np.abs(lg1[0] - lo1).max()), step1_tol=tol1, scale=float(np.abs(lo).max()),
           noise_prefill=float(np.abs(lo - ln).max()), noise_step1=float(np.abs(lo1 - ln1).max()))
    assert np.abs(lg[0] - lo).max() <= tol, (float(np.abs(lg[0] - lo).max()), tol)
    assert np.abs(lg1[0] - lo1).max() <= tol1, (float(np.abs(lg1[0] - lo1).max()), tol1)


@pytest.mark.timeout(900)
def test_full_configs3_f16_b64_30s(full, parity):
    """configs[3]'s per-GPU shape at full size: Qwen3-ASR-0.6B f16 (synthetic
    weights), 64 x 30 s clips (P = 405, 105-token budget) -- the skinny
    QKV / o / gate-up / down tilings at 64 rows, per-sequence decode attention
    over the exact kernels and the batched LM head.  All 64 rows bit-identical
    (identical clips), every budget met, row 0's prefill and 5 teacher-forced
    decode steps against the default oracle within 1e-2 of the logit scale
    (absolute |delta| printed)."""
    m, _, om = full
    B, n, budget = 64, 30 * SR, 105
    pcm = qasr.synth_pcm(17500, n)
    mel = op.log_mel(pcm)
    feats = om.encode(mel)
    ids, pos = m.build_prompt(feats.shape[0])
    assert len(ids) == 405
    d = op.OracleDecoder(om, len(ids) + 8)
    lo = [d.forward(ids, 0, feats, pos)]
    toks = [int(np.argmax(lo[0]))]
    for k in range(1, 6):
        lo.append(d.forward([toks[-1]], len(ids) + k - 1))
        toks.append(int(np.argmax(lo[-1])))
    c = qasr.Context(m, max_batch=B, max_ctx=len(ids) + budget + 8)
    try:
        assert c.get_option("fa_exact_decode") == 1
        r = c.transcribe([pcm] * B, max_tokens=budget, ignore_eos=True)
        assert all(len(t) == budget for t in r.tokens)
        assert all(t == r.tokens[0] for t in r.tokens)
        lg, am = c.prefill([ids] * B, [feats] * B, [pos] * B)
        for b in range(1, B):
            assert np.array_equal(lg[b], lg[0]), b
        errs = [_err(lg[0], lo[0])]
        for k in range(1, 6):
            lg, am = c.decode_step([toks[k - 1]] * B, [len(ids) + k - 1] * B)
            for b in range(1, B):
                assert np.array_equal(lg[b], lg[0]), (k, b)
            errs.append(_err(lg[0], lo[k]))
    finally:
        c.close()
    print("configs[3] prefill + decode steps (abs, rel):", [(round(a_, 4), round(r_, 5)) for a_, r_ in errs])
    parity("configs3_f16_b64_30s_row0_prefill_and_5_steps", abs_max=[e[0] for e in errs], rel_max=[e[1] for e in errs],
           scale=float(np.abs(lo[0]).max()))
    # measured abs <= 0.0226, rel <= 1.1e-3 (profiles/r4/parity.json): the bars above with ~2x margin
    assert max(r_ for _, r_ in errs) <= REL_LOGITS and max(a_ for a_, _ in errs) <= ABS_LOGITS, errs


def test_full_fx_seq_one_launch_bit_identical(full):
    """Decode batches on the per-sequence kernel run ggml's fp16-accumulating
    attention as one launch (option fx_seq: scores kept in LDS, then the
    chain) instead of a scores launch and a chain launch: the same arithmetic,
    so decode-step logits of a ragged 64-row batch (contexts 40..400 keys)
    are bit-identical with the option off."""
    m, _, _ = full
    B = 64
    rng = np.random.default_rng(23)
    lens = [40 + (b * 360) // (B - 1) for b in range(B)]
    rows = [[int(t) for t in rng.integers(0, 151643, n)] for n in lens]
    toks = [[int(t) for t in rng.integers(0, 151643, B)] for _ in range(3)]
    runs = {}
    for fx in (1, 0):
        c = qasr.Context(m, max_batch=B, max_ctx=420)
        try:
            c.set_option("fx_seq", fx)
            c.prefill(rows, want_logits=False)
            runs[fx] = [c.decode_step(t, [n + s for n in lens])[0].copy() for s, t in enumerate(toks)]
        finally:
            c.close()
    for s in range(len(toks)):
        assert np.isfinite(runs[1][s]).all()
        assert np.array_equal(runs[1][s], runs[0][s]), s


def test_full_skinny_inflight_bit_identical(full):
    """decode batches (9..64 rows): the skinny GEMMs with every K chunk of a
    wave in flight at once (option skinny_inf = 1, the default) multiply the
    same fragments in the same order as the one-chunk-at-a-time loop
    (skinny_inf = 0): logits bit-identical at 16 and 64 rows"""
    m, _, om = full
    feats = om.encode(op.log_mel(qasr.synth_pcm(18100, 2 * SR)))
    ids, pos = m.build_prompt(feats.shape[0])
    for B in (16, 64):
        c = qasr.Context(m, max_batch=B, max_ctx=len(ids) + 16)
        try:
            toks = [int(t) for t in np.random.default_rng(B).integers(0, 151643, B)]
            out = {}
            for inf in (1, 0):
                c.set_option("skinny_inf", inf)
                c.prefill([ids] * B, [feats] * B, [pos] * B, want_logits=False)
                lg, _ = c.decode_step(toks, [len(ids)] * B)
                out[inf] = lg
            assert np.array_equal(out[0], out[1]), (B, float(np.abs(out[0] - out[1]).max()))
        finally:
            c.close()


def test_full_q8_skinny_inflight_bit_identical(gpu, full_q8_gguf):
    """the Q8_0 skinny GEMMs (gemm_skinny_q8_kernel, CPW chunks in
    flight with hand-counted vmcnt waits) against the one-chunk loop
    (skinny_inf = 0) at 16 and 64 rows of the full-size Q8_0 model (K = 1024 /
    2048 / 3072: 1-3 chunks a wave): bit-identical decode-step logits."""
    m = qasr.Model(full_q8_gguf)
    try:
        rng = np.random.default_rng(31)
        ids = [int(t) for t in rng.integers(0, 151643, 40)]
        for B in (16, 64, 100):   # 100: the 65..128-row tilings
            c = qasr.Context(m, max_batch=B, max_ctx=64)
            try:
                toks = [int(t) for t in np.random.default_rng(B).integers(0, 151643, B)]
                out = {}
                for inf in (1, 0):
                    c.set_option("skinny_inf", inf)
                    c.prefill([ids] * B, want_logits=False)
                    lg, _ = c.decode_step(toks, [len(ids)] * B)
                    out[inf] = lg.copy()
                assert np.isfinite(out[1]).all()
                assert np.array_equal(out[0], out[1]), (B, float(np.abs(out[0] - out[1]).max()))
            finally:
                c.close()
    finally:
        m.close()


# Every per-context option that engine.hip's fuse_options() reads from the
# environment (QASR_<NAME>) and no other test switches: the value a user could
# set against the default, and what it must give.  "bits": the same arithmetic
# in another launch shape, schedule or prefetch -- decode-step logits, prefill
# logits and greedy tokens bit-identical to the default; "oracle": another
# arithmetic (the oracle switch named) within the decoder bars.  Batch-1
# options run on a 1-row context (the fused launches), batch options on 16 rows.
OPTION_CASES = {
    "ffn_delay": (0, "bits", 1), "ffn_wdelay": (0, "bits", 1), "qkv_delay": (0, "bits", 1), "o_delay": (0, "bits", 1),
    "handoff_fence": (1, "bits", 1), "gran": (0, "bits", 1), "att_spl1": (128, "bits", 1),
    "fx_vpf": (0, "bits", 1), "fx_vpf=1": (1, "bits", 1), "fx_vpf=3": (3, "bits", 1),
    "fa_exact_prefill": (0, "oracle", 1),
    "att_spl": (128, "bits", 16), "lmh": (0, "bits", 16), "skinny": (0, "oracle", 16),
    "lmh@100": (0, "bits", 100),   # 65..128 rows: the one-launch LM head (lmhead128_kernel) against the separate launches
    "skinny@100": (0, "oracle", 100),   # 65..128 rows: the skinny GEMMs' 128-row tilings (default) and the tiled GEMMs
    "skinny_wdef": (0, "bits", 16), "skinny_wdef@100": (0, "bits", 100),   # weights nontemporal (default: cache policy)
}


@pytest.mark.parametrize("case", list(OPTION_CASES))
def test_full_option_matches_default(full, case):
    m, _, om = full
    name = case.split("=")[0].split("@")[0]
    val, kind, B = OPTION_CASES[case]
    pcm = qasr.synth_pcm(19000, 2 * SR)
    feats = om.encode(op.log_mel(pcm))
    ids, pos = m.build_prompt(feats.shape[0])
    c = qasr.Context(m, max_batch=B, max_ctx=160)
    try:
        def run():
            lp, _ = c.prefill([ids] * B, [feats] * B, [pos] * B)
            lp = lp.copy()
            lg, _ = c.decode_step([1234] * B, [len(ids)] * B)
            toks = c.transcribe([pcm] * B, max_tokens=8, ignore_eos=True).tokens
            return lp, lg.copy(), toks
        base = run()
        c.set_option(name, val)
        assert c.get_option(name) == val
        alt = run()
    finally:
        c.close()
    if kind == "bits":
        assert np.array_equal(base[0], alt[0]) and np.array_equal(base[1], alt[1]), case
        assert base[2] == alt[2], case
    else:
        # the option's run against the oracle (prefill rows and the decode step's rows), and the
        # default's decode rows too: the default path differs from the option's only there
        flags = op.OracleModel.FA_V_F32 if name == "fa_exact_prefill" else 0
        d = op.OracleDecoder(om, 160, flags)
        lo = d.forward(ids, 0, feats, pos)
        ld = d.forward([1234], len(ids))
        for b in range(B):
            ab, rel = _err(alt[0][b], lo)
            assert rel <= REL_LOGITS and ab <= ABS_LOGITS, (case, b, ab, rel)
            if name != "fa_exact_prefill":
                for run in (base, alt):
                    ab, rel = _err(run[1][b], ld)
                    assert rel <= REL_LOGITS and ab <= ABS_LOGITS, (case, "decode", b, ab, rel)
        assert all(t == alt[2][0] for t in alt[2])
        assert all(t == base[2][0] for t in base[2])


@pytest.mark.timeout(900)
def test_full_stream_34_slots_refills_across_split_buckets(full):
    """continuous batching at full size with more than 8
    slots -- 34 slots take the decode-batch kernels (skinny GEMMs, the
    one-launch LM head, the per-sequence exact attention indexed by slot) --
    48 clips of 2-19 s with ragged budgets, so refills land mid-stream and
    several clips' contexts cross a 256-key split bucket (prompt < 256 <=
    prompt + budget).  Every clip's tokens equal the same clip's in a static
    batch of 34 clips (the same decode kernels, run to the batch's longest
    budget and truncated): a clip's result depends neither on its slot nor on
    when the slot was refilled."""
    m, _, _ = full
    S, n = 34, 48
    rng = np.random.default_rng(77)
    secs = rng.uniform(2.0, 19.0, n)
    secs[:4] = [18.0, 17.5, 17.9, 2.0]   # prompts 249, 243, 248: each crosses 256 within its budget
    lens = [int(s * 100) * 160 for s in secs]
    budgets = [int(b) for b in rng.integers(3, 28, n)]
    budgets[:3] = [27, 20, 26]
    prompts = [qasr.lib().qasr_prompt_len(qasr.encoder_frames(qasr.mel_frames(L))) for L in lens]
    assert sum(P < 256 <= P + b for P, b in zip(prompts, budgets)) >= 2
    clips = [qasr.synth_pcm(7600 + i, L) for i, L in enumerate(lens)]
    c = qasr.Context(m, max_batch=S, max_ctx=max(prompts) + max(budgets) + 8)
    try:
        it = iter([(i, clips[i], budgets[i]) for i in range(n)])
        out, st = c.run_stream(lambda: next(it, None), max_tokens=max(budgets), ignore_eos=True)
        assert st.n_clips == n and st.n_errors == 0 and st.n_prefills >= 2
        ref = {}
        for k in range(0, n, S):
            idx = list(range(k, min(k + S, n)))
            pad = [i for i in range(n) if i not in idx][:S - len(idx)]   # a full batch: the same kernels as the stream
            r = c.transcribe([clips[i] for i in idx + pad], max_tokens=max(budgets[i] for i in idx), ignore_eos=True)
            for j, i in enumerate(idx):
                ref[i] = r.tokens[j][:budgets[i]]
    finally:
        c.close()
    for i in range(n):
        assert len(out[i]) == budgets[i] and out[i] == ref[i], i
