"""CPU: the oracle's encoder/decoder restatement on the tiny synthetic model --
self-consistency properties the reference's graphs have by construction."""
import numpy as np
import pytest

import oracle_py as op
import qasr


@pytest.fixture(scope="module")
def om(tiny_oracle):
    return tiny_oracle


def test_encoder_shapes_and_chunking(om):
    """per-100-frame chunks, short last chunk not padded (src/audio_encoder.cpp:331-343)"""
    for n in [16000, 16000 + 160 * 37, 3 * 16000]:
        mel = op.log_mel(qasr.synth_pcm(1, n))
        f = om.encode(mel)
        assert f.shape == (qasr.encoder_frames(mel.shape[1]), om.hidden)
        assert np.isfinite(f).all()


def test_conv_chunks_are_independent(om):
    """each chunk's conv stack sees only its own 100 frames, PE restarts at 0:
    encoding frames [0,200) equals concatenating encodes of [0,100) and [100,200)."""
    mel = op.log_mel(qasr.synth_pcm(2, 2 * 16000 + 400))[:, :200]
    whole = om.encode_conv(np.ascontiguousarray(mel))
    a = om.encode_conv(np.ascontiguousarray(mel[:, :100]))
    b = om.encode_conv(np.ascontiguousarray(mel[:, 100:]))
    assert np.array_equal(whole, np.concatenate([a, b]))


def test_prefill_equals_incremental(om):
    mel = op.log_mel(qasr.synth_pcm(3, 16000))
    feats = om.encode(mel)
    ids = om.prompt(feats.shape[0])
    d1 = op.OracleDecoder(om, 256)
    l1 = d1.forward(ids, 0, feats, 9)
    d2 = op.OracleDecoder(om, 256)
    d2.forward(ids[:-4], 0, feats, 9)
    for i in range(4):
        l2 = d2.forward(ids[len(ids) - 4 + i:len(ids) - 3 + i], len(ids) - 4 + i)
    assert np.array_equal(l1, l2)


def test_numerics_switches_are_small(om):
    """ggml's fp16 GELU table and fp16 FA V-accumulator vs exact variants:
    differences stay far below the stated tolerances."""
    mel = op.log_mel(qasr.synth_pcm(4, 16000))
    a = om.encode(mel)
    b = om.encode(mel, om.GELU_EXACT)
    assert 0 < np.abs(a - b).max() < 2e-2
    ids = om.prompt(a.shape[0])
    la = op.OracleDecoder(om, 128, 0).forward(ids, 0, a, 9)
    lb = op.OracleDecoder(om, 128, om.FA_V_F32).forward(ids, 0, a, 9)
    assert np.abs(la - lb).max() <= 1e-2 * np.abs(la).max()


def test_greedy_loop_rules(om):
    pcm = qasr.synth_pcm(5, 16000)
    t1, _ = om.transcribe(pcm, max_tokens=12, ignore_eos=True)
    t2, _ = om.transcribe(pcm, max_tokens=12, ignore_eos=True)
    assert t1 == t2 and len(t1) == 12
    t3, _ = om.transcribe(pcm, max_tokens=12, ignore_eos=False)
    assert len(t3) <= 12 and 151645 not in t3
    assert om.transcribe(qasr.synth_pcm(6, 100), max_tokens=4)[0] == []   # no audio frames -> error path


def test_argmax_tie_rule(built):
    x = np.zeros(16, np.float32)
    x[[3, 7, 11]] = 5.0
    assert op.olib().qo_argmax(op._f(x), 16) == 3
