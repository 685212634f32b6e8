"""Structural anchor of the encoder/decoder restatement: transformers'
independent qwen3_asr implementation, loaded with the tiny synthetic GGUF's
weights (tests/golden/make_hf_anchor.py wrote the fixture).

Pins the GGUF name/transpose map, conv feature order c*16+f, per-chunk PE
restart, projector, NEOX RoPE, q/k norm, GQA, audio splice and tied LM head
-- not ggml's numerics (HF is fp32; ggml rounds matmul inputs to fp16, which
the oracle restates), hence a tolerance: measured oracle vs HF on the three
clips 1.3e-3 max |feature diff| at a feature scale of 2 (6.5e-4 relative) and
0.025 max |logit diff| at a logit scale of 21-24 (1.2e-3 relative).  A
structural slip (a transposed weight, a wrong feature order, RoPE pairs i/i+1
instead of i/i+64, a missing PE restart) moves these by O(1).
"""
import os

import numpy as np
import pytest

import oracle_py as op
import qasr

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "hf_anchor.npz")
FEAT_TOL = 2.5e-3   # x max |feature|
LOGIT_TOL = 2.5e-3  # x max |logit|


@pytest.fixture(scope="module")
def anchor():
    return np.load(FIX)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_oracle_matches_hf_structure(tiny_oracle, anchor, i):
    mel = anchor[f"mel{i}"]
    assert np.array_equal(mel, op.log_mel(qasr.synth_pcm(21000 + i, mel.shape[1] * 160)))
    feats = tiny_oracle.encode(mel)
    hf = anchor[f"feats{i}"]
    assert feats.shape == hf.shape
    assert np.abs(feats - hf).max() <= FEAT_TOL * np.abs(hf).max()
    ids = anchor[f"ids{i}"]
    assert np.array_equal(ids, tiny_oracle.prompt(feats.shape[0]))
    lo = op.OracleDecoder(tiny_oracle, 256).forward(ids, 0, feats, 9)
    scale = float(anchor[f"logits_absmax{i}"])
    assert np.abs(lo[:4096] - anchor[f"logits_head{i}"]).max() <= LOGIT_TOL * scale
    top = anchor[f"logits_top_idx{i}"]
    assert np.abs(lo[top] - anchor[f"logits_top_val{i}"]).max() <= LOGIT_TOL * scale
    assert int(np.argmax(lo)) == int(top[0])


@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 2])
def test_gpu_matches_hf_structure(gpu, tiny_gguf, anchor, i):
    """The HIP path against the same independent implementation."""
    m = qasr.Model(tiny_gguf)
    c = qasr.Context(m, max_batch=1, max_ctx=256)
    try:
        mel = anchor[f"mel{i}"]
        feats = c.encode([mel])[0]
        hf = anchor[f"feats{i}"]
        assert np.abs(feats - hf).max() <= FEAT_TOL * np.abs(hf).max()
        ids = anchor[f"ids{i}"]
        lg, am = c.prefill([ids], [feats], [9])
        scale = float(anchor[f"logits_absmax{i}"])
        assert np.abs(lg[0][:4096] - anchor[f"logits_head{i}"]).max() <= LOGIT_TOL * scale
        assert int(am[0]) == int(anchor[f"logits_top_idx{i}"][0])
    finally:
        c.close()
        m.close()
