"""GPU parity of the forced-aligner path (BASELINE config 5) through the C-ABI
against the oracle's aligner restatement (src/forced_aligner.cpp:591-1306).

Tolerances: encoder as the ASR encoder (max 2e-2, mean 1e-3 -- the
reference's own tests/run_all_tests.sh:166); timestamp classes identical
wherever the oracle's own top-1/top-2 margin exceeds its noise floor (0.5 % of
the logit scale: the summation orders of the fp32 dots differ).  The prefill
attention follows the reference's: Q and K in fp32 (fp32 MFMA scores), V cast
to fp16 and accumulated in fp16 key by key (src/forced_aligner.cpp:1041-1046,
csrc/fa_exact.hip)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as op
import qasr

pytestmark = pytest.mark.gpu
SR = 16000
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "qwen3-asr.cpp_amd", "qwen3-asr-cli")


@pytest.fixture(scope="module")
def al(gpu, tmp_path_factory):
    p = str(tmp_path_factory.mktemp("alg") / "aligner-tiny.gguf")
    qasr.write_synthetic_gguf(p, "aligner-tiny", 42, 1)
    op.set_threads(min(16, os.cpu_count() or 1))
    om = op.OracleModel(p)
    m = qasr.Model(p)
    c = qasr.Context(m, max_batch=1, max_ctx=2048)
    yield p, m, c, om
    c.close()
    m.close()


def _stats(a, b):
    d = np.abs(a - b)
    return float(d.max()), float(d.mean())


@pytest.mark.parametrize("secs", [0.7, 2.3, 9.5, 10.0, 13.37])
def test_aligner_encode_matches_oracle(al, secs):
    _, _, c, om = al
    mel = op.log_mel(qasr.synth_pcm(8100, int(secs * SR)))
    g = c.encode([mel])[0]
    o = om.encode(mel)
    assert g.shape == o.shape
    mx, mean = _stats(g, o)
    assert mx <= 2e-2 and mean <= 1e-3, (mx, mean)


def test_aligner_windows_on_gpu(al):
    _, _, c, _ = al
    mel = op.log_mel(qasr.synth_pcm(8200, SR * 11 + 3210))
    a = c.encode([mel])[0]
    mel2 = mel.copy()
    mel2[:, 800:] += 1.0
    b = c.encode([mel2])[0]
    assert np.array_equal(a[:104], b[:104]) and not np.array_equal(a[104:], b[104:])


@pytest.mark.parametrize("secs,text", [(2.0, "ab cd ef"), (6.4, "ab cd ef gh ij kl mn op qr st"), (10.0, "xy zz ab")])
def test_aligner_classes_match_oracle(al, secs, text):
    _, m, c, om = al
    pcm = qasr.synth_pcm(8300 + int(secs * 10), int(secs * SR))
    ids, nw = m.align_tokenize(text)
    cls, t = c.align(pcm, ids)
    ocls, olg, _ = om.align_classes(pcm, ids)
    assert len(cls) == len(ocls) == 2 * nw
    scale = float(np.abs(olg).max())
    srt = np.sort(olg, axis=1)
    margin = srt[:, -1] - srt[:, -2]
    same = np.array(cls) == np.array(ocls)
    assert same[margin > 5e-3 * scale].all(), (cls, ocls, margin / scale)
    assert same.all(), (cls, ocls, margin / scale)   # measured: every row, these seeds (no near-ties)
    assert t.t_encode_ms > 0 and t.t_total_ms > 0


def test_align_json_document(al):
    _, m, c, _ = al
    pcm = qasr.synth_pcm(8400, int(3.3 * SR))
    text = 'ab "cd" e\\f gh'
    doc, _ = c.align_json(pcm, text)
    words = doc["words"]
    assert [w["word"] for w in words] == text.split()
    ids, _ = m.align_tokenize(text)
    cls, _ = c.align(pcm, ids)
    fixed = qasr.fix_timestamps(cls)
    dur = np.float32(len(pcm) / SR)
    ts = [min(np.float32(k) * np.float32(0.08), dur) for k in fixed]
    for i, w in enumerate(words):
        assert w["start"] == pytest.approx(float(ts[2 * i]), abs=5e-4)
        assert w["end"] == pytest.approx(float(ts[2 * i + 1]), abs=5e-4)
        assert 0 <= w["start"] <= dur + 1e-3 and 0 <= w["end"] <= dur + 1e-3
    # LIS-repaired classes are non-decreasing whenever the repair interpolates
    assert all(isinstance(w["start"], float) for w in words)


def test_align_errors(al, gpu, tiny_gguf):
    _, _, c, _ = al
    with pytest.raises(qasr.QasrError):
        c.align(np.zeros(0, np.float32), [TS := 151705])
    m = qasr.Model(tiny_gguf)   # an ASR model has no classification head
    ca = qasr.Context(m, 1, 256)
    try:
        with pytest.raises(qasr.QasrError, match="ForcedAligner"):
            ca.align(qasr.synth_pcm(1, SR), [TS])
    finally:
        ca.close()
        m.close()


def test_cli_align_and_transcribe_align(al, tiny_gguf, tmp_path):
    p, _, _, _ = al
    wav = str(tmp_path / "a.wav")
    qasr.write_wav(wav, qasr.synth_pcm(8500, int(2.5 * SR)))
    out = str(tmp_path / "o.json")
    r = subprocess.run([CLI, "-m", p, "-f", wav, "--align", "--text", "ab cd ef", "-o", out, "--no-timing"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    import json
    doc = json.load(open(out))
    assert [w["word"] for w in doc["words"]] == ["ab", "cd", "ef"]
    r = subprocess.run([CLI, "-m", tiny_gguf, "--aligner-model", p, "-f", wav, "-a", "--max-tokens", "12"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert '"words"' in r.stdout and "Phase 2: Forced Alignment" in r.stderr


@pytest.mark.slow
def test_full_aligner_encode_and_classes(gpu, tmp_path_factory, parity):
    """Qwen3-ForcedAligner-0.6B dimensions (24 x 1024 encoder, vocab 152064)."""
    p = str(tmp_path_factory.mktemp("alf") / "aligner-full.gguf")
    qasr.write_synthetic_gguf(p, "aligner", 42, 1)
    om = op.OracleModel(p)
    m = qasr.Model(p)
    c = qasr.Context(m, 1, 1024)
    try:
        assert (m.hp.enc_layers, m.hp.d_model, m.hp.enc_heads, m.hp.enc_ffn, m.hp.vocab_size) == (24, 1024, 16, 4096, 152064)
        pcm = qasr.synth_pcm(8600, int(1.6 * SR))
        mel = op.log_mel(pcm)
        mx, mean = _stats(c.encode([mel])[0], om.encode(mel))
        assert mx <= 2e-2 and mean <= 1e-3, (mx, mean)
        ids, nw = m.align_tokenize("ab cd")
        cls, _ = c.align(pcm, ids)
        ocls, olg, _ = om.align_classes(pcm, ids)
        scale = float(np.abs(olg).max())
        srt = np.sort(olg, axis=1)
        margin = srt[:, -1] - srt[:, -2]
        same = np.array(cls) == np.array(ocls)
        parity("full_aligner_1p6s", enc_abs_max=mx, enc_abs_mean=mean, rows=len(cls), classes_equal=int(same.sum()),
               min_margin_rel=float((margin / scale).min()), mismatch_margins_rel=(margin / scale)[~same].tolist())
        assert same[margin > 5e-3 * scale].all(), (cls, ocls, margin / scale)
    finally:
        c.close()
        m.close()


def test_align_json_batch_equals_single(al):
    """qasr_align_json_batch (configs[4]'s aligner leg over many transcripts):
    clips of different lengths and texts in one aligner pass give the same
    documents as one clip at a time, and the classes match the oracle's"""
    p, m, _, om = al
    clips = [qasr.synth_pcm(8500 + i, int(s * SR)) for i, s in enumerate((2.0, 6.4, 0.9, 10.0))]
    texts = ["ab cd ef", "ab cd ef gh ij kl mn op", "xy", 'zz "q" ab']
    cb = qasr.Context(m, max_batch=4, max_ctx=2048)
    try:
        docs, t = cb.align_json_batch(clips, texts)
        assert t.t_total_ms > 0
        for pcm, text, d in zip(clips, texts, docs):
            one, _ = cb.align_json(pcm, text)
            assert d == one
        ids, _ = m.align_tokenize(texts[1])
        cls, _ = cb.align(clips[1], ids)
        ocls, olg, _ = om.align_classes(clips[1], ids)
        srt = np.sort(olg, axis=1)
        margin = srt[:, -1] - srt[:, -2]
        same = np.array(cls) == np.array(ocls)
        assert same[margin > 5e-3 * float(np.abs(olg).max())].all(), (cls, ocls)
        with pytest.raises(qasr.QasrError):   # more clips than the context's slots
            cb.align_json_batch(clips + clips[:1], texts + texts[:1])
    finally:
        cb.close()
