"""GPU parity: the HIP path (through the C-ABI, libqasr.so) against the CPU
oracle (oracle/qasr_oracle.c) on the same seeded inputs.

Tolerances (stated per test) follow the reference's own: mel 1e-4
(tests/run_all_tests.sh:134), encoder 2e-2 (tests/run_all_tests.sh:166,
tests/test_encoder.cpp:157), decoder logits 1e-2 relative to the logit scale
(tests/test_decoder.cpp:157).  Greedy token ids must be identical; where the
oracle's own top-1/top-2 margin at a step is below the numeric noise floor the
comparison is margin-aware (first-divergence index + margin reported).
"""
import numpy as np
import pytest

import oracle_py as op
import qasr

pytestmark = pytest.mark.gpu

SR = 16000


@pytest.fixture(scope="module")
def tiny(gpu, tiny_gguf):
    m = qasr.Model(tiny_gguf)
    c = qasr.Context(m, max_batch=4, max_ctx=640)
    yield m, c
    c.close()
    m.close()


def test_prefill_expf_replacement_is_bit_exact(gpu):
    """fa_exact.hip's exact prefill attention takes its weights through
    px_expf_nonpos (the device expf's instruction sequence without the overflow
    clamp, round 6): on every non-positive fp32 input its result must be the
    device expf's bits, so the kernel's (ms, vs) stay the round-5 kernel's"""
    import ctypes
    bad = ctypes.c_uint64(12345)
    assert qasr.lib().qasr_check_expf_nonpos(0, ctypes.byref(bad)) == 0, qasr.lib().qasr_last_error()
    assert bad.value == 0, bad.value


# ------------------------------------------------------------------ mel
@pytest.mark.parametrize("n", [0, 1, 159, 160, 161, 401, SR, int(2.5 * SR), int(7.3 * SR)])
def test_mel_matches_oracle(tiny, n):
    _, c = tiny
    pcm = qasr.synth_pcm(1000 + n, n)
    g = c.mel([pcm])[0]
    o = op.log_mel(pcm)
    assert g.shape == o.shape == (128, n // 160)
    if o.size:
        err = np.abs(g - o).max()
        assert err <= 1e-5, err                      # reference tolerance 1e-4 / 1e-5
        assert (g == o).mean() > 0.999               # fp64 DFT replays the reference's FMA chain


def test_mel_batch_ragged(tiny):
    _, c = tiny
    lens = [SR, 3 * SR + 77, 250, 2 * SR]
    clips = [qasr.synth_pcm(2000 + i, n) for i, n in enumerate(lens)]
    gs = c.mel(clips)
    for pcm, g in zip(clips, gs):
        o = op.log_mel(pcm)
        assert g.shape == o.shape
        if o.size:
            assert np.abs(g - o).max() <= 1e-5


# -------------------------------------------------------------- encoder
def _stats(a, b):
    d = np.abs(a - b)
    return float(d.max()), float(d.mean())


@pytest.mark.parametrize("secs", [0.5, 1.0, 2.37, 4.0])
def test_encode_conv_matches_oracle(tiny, tiny_oracle, secs):
    _, c = tiny
    pcm = qasr.synth_pcm(3000, int(secs * SR))
    mel = op.log_mel(pcm)
    g = c.encode_conv([mel])[0]
    o = tiny_oracle.encode_conv(mel)
    assert g.shape == o.shape
    mx, mean = _stats(g, o)
    assert mx <= 2e-2 and mean <= 1e-3, (mx, mean)


@pytest.mark.parametrize("secs", [0.5, 1.0, 2.37, 9.5])
def test_encode_matches_oracle(tiny, tiny_oracle, secs):
    _, c = tiny
    pcm = qasr.synth_pcm(4000, int(secs * SR))
    mel = op.log_mel(pcm)
    g = c.encode([mel])[0]
    o = tiny_oracle.encode(mel)
    assert g.shape == o.shape
    mx, mean = _stats(g, o)
    assert mx <= 2e-2 and mean <= 1e-3, (mx, mean)


@pytest.mark.parametrize("secs", [2.37, 12.3])
def test_encoder_attention_paths_match_oracle(tiny, tiny_oracle, secs):
    """Encoder attention on split fp16 operands (the default) and on fp32 MFMA
    (option enc_attn_f32): both within the fp32 encoder bar of the oracle, the
    split path no further from it than the fp32 one (the two differ by fp16
    rounding flips of the attention output that feeds the o-projection)."""
    _, c = tiny
    mel = op.log_mel(qasr.synth_pcm(4100, int(secs * SR)))
    o = tiny_oracle.encode(mel)
    try:
        c.set_option("enc_attn_f32", 1)
        g32 = c.encode([mel])[0]
    finally:
        c.set_option("enc_attn_f32", 0)
    g = c.encode([mel])[0]
    mx, mean = _stats(g, o)
    mx32, mean32 = _stats(g32, o)
    assert mx <= 2e-2 and mean <= 1e-3, (mx, mean)
    assert mx32 <= 2e-2 and mean32 <= 1e-3, (mx32, mean32)
    assert mean <= 1.25 * mean32 + 1e-5 and mx <= 1.5 * mx32 + 1e-3, (mx, mean, mx32, mean32)


def test_encode_batch_equals_single(tiny):
    _, c = tiny
    mels = [op.log_mel(qasr.synth_pcm(5000 + i, n)) for i, n in enumerate([SR, 3 * SR + 500, 2 * SR - 7])]
    batched = c.encode(mels)
    for m_, b in zip(mels, batched):
        s = c.encode([m_])[0]
        assert np.array_equal(s, b)


# -------------------------------------------------------------- decoder
def test_prefill_logits_match_oracle(tiny, tiny_oracle):
    m, c = tiny
    pcm = qasr.synth_pcm(6000, 2 * SR)
    mel = op.log_mel(pcm)
    feats = tiny_oracle.encode(mel)
    ids, pos = m.build_prompt(feats.shape[0])
    assert np.array_equal(ids, tiny_oracle.prompt(feats.shape[0])) and pos == 9
    lg, am = c.prefill([ids], [feats], [pos])
    d = op.OracleDecoder(tiny_oracle, 512)
    lo = d.forward(ids, 0, feats, pos)
    scale = float(np.abs(lo).max())
    assert np.abs(lg[0] - lo).max() <= 1e-2 * scale, (float(np.abs(lg[0] - lo).max()), scale)
    assert am[0] == int(np.argmax(lg[0]))
    top2 = np.sort(lo)[-2:]
    if top2[1] - top2[0] > 0.05:
        assert am[0] == op.olib().qo_argmax(op._f(lo), len(lo))


@pytest.mark.parametrize("exact", [1, 0])
def test_decode_steps_teacher_forced(tiny, tiny_oracle, exact, parity):
    """exact = 1 (the default): ggml's fp16 V accumulation (fx_chain.h),
    against the default oracle; exact = 0 (option fa_exact_decode = 0): the
    fp32-accumulating split-K decode attention, against the oracle's
    QO_FA_V_F32 switch (the same change made on the oracle side)"""
    m, c = tiny
    rng = np.random.default_rng(7)
    pcm = qasr.synth_pcm(6100, SR)
    feats = tiny_oracle.encode(op.log_mel(pcm))
    ids, pos = m.build_prompt(feats.shape[0])
    c.set_option("fa_exact_decode", exact)
    try:
        c.prefill([ids], [feats], [pos], want_logits=False)
        d = op.OracleDecoder(tiny_oracle, 512, 0 if exact else op.OracleModel.FA_V_F32)
        d.forward(ids, 0, feats, pos)
        n_past = len(ids)
        worst, worst_abs = 0.0, 0.0
        for step in range(24):
            tok = int(rng.integers(0, 151643))
            lg, am = c.decode_step([tok], [n_past])
            lo = d.forward([tok], n_past)
            scale = float(np.abs(lo).max())
            worst_abs = max(worst_abs, float(np.abs(lg[0] - lo).max()))
            worst = max(worst, float(np.abs(lg[0] - lo).max()) / scale)
            s = np.sort(lo)
            if s[-1] - s[-2] > 0.05 * scale:
                assert am[0] == int(np.argmax(lo)), step
            n_past += 1
    finally:
        c.set_option("fa_exact_decode", 1)   # the default
    parity(f"tiny_decode_24_steps_exact{exact}", abs_max=worst_abs, rel_max=worst)
    # measured 0.012 / 0.017 absolute (6.6e-4 / 9.8e-4 of the scale): bars with ~2x margin
    assert worst <= 3e-3 and worst_abs <= 4e-2, (worst_abs, worst)


def _margin_aware_equal(gpu_toks, ora_toks, om, pcm, max_tokens, flags=0):
    """Token-exact unless the oracle's own top-1/top-2 margin at the first
    divergence is within the fp noise floor; returns (first_div, margin)."""
    n = min(len(gpu_toks), len(ora_toks))
    first = next((i for i in range(n) if gpu_toks[i] != ora_toks[i]), None)
    if first is None:
        assert len(gpu_toks) == len(ora_toks)
        return None, None
    # replay the oracle to the divergence and measure its margin there
    mel = op.log_mel(pcm)
    feats = om.encode(mel)
    ids = om.prompt(feats.shape[0])
    d = op.OracleDecoder(om, len(ids) + max_tokens + 1, flags)
    lo = d.forward(ids, 0, feats, 9)
    for i in range(first):
        lo = d.forward([ora_toks[i]], len(ids) + i)
    s = np.sort(lo)
    margin = float(s[-1] - s[-2])
    assert margin <= 2e-2 * float(np.abs(lo).max()), (first, margin)
    return first, margin


def test_transcribe_matches_oracle(tiny, tiny_oracle):
    _, c = tiny
    for i, secs in enumerate([1.0, 3.3]):
        pcm = qasr.synth_pcm(7000 + i, int(secs * SR))
        r = c.transcribe([pcm], max_tokens=32, ignore_eos=True)
        ora, _ = tiny_oracle.transcribe(pcm, max_tokens=32, ignore_eos=True)
        assert len(r.tokens[0]) == 32
        _margin_aware_equal(r.tokens[0], ora, tiny_oracle, pcm, 32)


def test_transcribe_batch_equals_single(tiny):
    _, c = tiny
    clips = [qasr.synth_pcm(8000 + i, n) for i, n in enumerate([SR, 2 * SR + 333, 4 * SR])]
    rb = c.transcribe(clips, max_tokens=16, ignore_eos=True)
    for pcm, tb in zip(clips, rb.tokens):
        rs = c.transcribe([pcm], max_tokens=16, ignore_eos=True)
        assert rs.tokens[0] == tb


def test_transcribe_eos_and_errors(tiny):
    m, c = tiny
    r = c.transcribe([qasr.synth_pcm(9000, SR)], max_tokens=8, ignore_eos=False)
    assert len(r.tokens[0]) <= 8
    assert 151645 not in r.tokens[0]            # trailing EOS popped, never emitted mid-sequence
    with pytest.raises(qasr.QasrError, match="audio_pad"):
        c.transcribe([qasr.synth_pcm(9001, 100)], max_tokens=4)   # < 160 samples: no audio frames
    with pytest.raises(qasr.QasrError, match="Context length"):
        c.transcribe([qasr.synth_pcm(9002, SR)], max_tokens=10000)


def test_chunk_prefill_after_cached_tokens(tiny, tiny_oracle, parity):
    """TextDecoder::forward with n_tokens > 1 at n_past > 0 (src/text_decoder.cpp:
    392-581: one causal graph for the chunk) = qasr_prefill_chunk: the chunk's
    last-row logits, and a decode step after it, against the oracle's chunk
    forward; two chunks back to back, then a chunk at n_past = 0"""
    m, c = tiny
    feats = tiny_oracle.encode(op.log_mel(qasr.synth_pcm(6300, SR)))
    ids, pos = m.build_prompt(feats.shape[0])
    c.prefill([ids], [feats], [pos], want_logits=False)
    d = op.OracleDecoder(tiny_oracle, 512)
    d.forward(ids, 0, feats, pos)
    rng = np.random.default_rng(13)
    n_past, errs = len(ids), []
    for n in (5, 17):
        chunk = [int(t) for t in rng.integers(0, 151643, n)]
        lg, am = c.prefill_chunk([chunk], [n_past])
        lo = d.forward(chunk, n_past)
        errs.append(float(np.abs(lg[0] - lo).max()) / float(np.abs(lo).max()))
        assert errs[-1] <= 1e-2, errs
        n_past += n
    tok = int(rng.integers(0, 151643))
    lg, _ = c.decode_step([tok], [n_past])
    lo = d.forward([tok], n_past)
    errs.append(float(np.abs(lg[0] - lo).max()) / float(np.abs(lo).max()))
    parity("tiny_chunk_prefill_5_17_then_step", rel_max=errs)
    assert errs[-1] <= 1e-2, errs
    chunk = [int(t) for t in rng.integers(0, 151643, 9)]
    lg, _ = c.prefill_chunk([chunk], [0])
    d0 = op.OracleDecoder(tiny_oracle, 64)
    lo = d0.forward(chunk, 0)
    assert float(np.abs(lg[0] - lo).max()) <= 1e-2 * float(np.abs(lo).max())


def test_forward_with_audio_after_cached_tokens(tiny, tiny_oracle, parity):
    """TextDecoder::forward_with_audio at n_past > 0 (src/text_decoder.cpp:588-644;
    the splice of :431-459 applies to the chunk's own rows) = qasr_prefill_chunk_audio:
    the prompt's text head prefilled first (n_past = 0, no audio), then the rest
    of the prompt as one chunk with the audio rows spliced at their offset in the
    chunk, and a decode step -- against the oracle doing the same two calls, and
    the chunked result against the one-shot prefill"""
    m, c = tiny
    feats = tiny_oracle.encode(op.log_mel(qasr.synth_pcm(6400, int(1.7 * SR))))
    ids, pos = m.build_prompt(feats.shape[0])
    k = pos - 2   # the head stops two tokens before the audio pads
    d = op.OracleDecoder(tiny_oracle, 512)
    lg0, _ = c.prefill([ids[:k]])
    lo0 = d.forward(ids[:k], 0)
    lg1, am = c.prefill_chunk([ids[k:]], [k], feats_list=[feats], audio_pos=[pos - k])
    lo1 = d.forward(ids[k:], k, feats, pos - k)
    tok = int(am[0])
    lg2, _ = c.decode_step([tok], [len(ids)])
    lo2 = d.forward([tok], len(ids))
    errs = [float(np.abs(g[0] - o).max()) / float(np.abs(o).max()) for g, o in ((lg0, lo0), (lg1, lo1), (lg2, lo2))]
    parity("tiny_forward_with_audio_at_n_past", rel_max=errs)
    assert max(errs) <= 1e-2, errs
    assert tok == int(np.argmax(lo1))
    full, _ = c.prefill([ids], [feats], [pos])   # the same prompt in one call: the same rows up to rounding
    assert float(np.abs(full[0] - lg1[0]).max()) <= 1e-2 * float(np.abs(lo1).max())


@pytest.mark.parametrize("secs", [0.9, 3.1, 9.5])
def test_encode_no_chunk_matches_oracle(tiny, tiny_oracle, secs):
    """AudioEncoder::encode_no_chunk (src/audio_encoder.cpp:603-852): the conv
    stack over every frame as one chunk and PE positions 0..N-1, against the
    oracle's QO_ENC_NO_CHUNK at the encoder bar; up to 100 frames it equals encode"""
    _, c = tiny
    mel = op.log_mel(qasr.synth_pcm(6500, int(secs * SR)))
    g = c.encode_no_chunk([mel])[0]
    o = tiny_oracle.encode(mel, op.OracleModel.ENC_NO_CHUNK)
    assert g.shape == o.shape
    mx, mean = _stats(g, o)
    assert mx <= 2e-2 and mean <= 1e-3, (mx, mean)
    if mel.shape[1] <= 100:
        assert np.array_equal(g, c.encode([mel])[0])
