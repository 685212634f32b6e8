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


def test_encode_no_chunk_structure(om):
    """QO_ENC_NO_CHUNK (AudioEncoder::encode_no_chunk, src/audio_encoder.cpp:603-852):
    up to 100 frames it is the chunked encoder itself; past 100 the conv stack
    sees across chunk edges and the PE keeps counting, so the rows differ from
    the chunked ones after the first chunk but not before its edge region."""
    mel = op.log_mel(qasr.synth_pcm(7, 16000))   # 100 frames: one chunk
    assert np.array_equal(om.encode_conv(mel), om.encode_conv(mel, om.ENC_NO_CHUNK))
    mel = op.log_mel(qasr.synth_pcm(8, 3 * 16000 + 480))   # 303 frames
    a, b = om.encode_conv(mel), om.encode_conv(mel, om.ENC_NO_CHUNK)
    assert b.shape == (om.frames(303, om.ENC_NO_CHUNK), om.m.d_model) == (38, om.m.d_model) and a.shape[0] == 40
    assert np.array_equal(a[:12], b[:12])          # rows whose receptive field stays inside chunk 0
    assert not np.allclose(a[13:20], b[13:20])     # PE position 13.. vs the restarted 0..
    f = om.encode(mel, om.ENC_NO_CHUNK)
    assert f.shape == (38, om.hidden) and np.isfinite(f).all()
