"""CPU: boundary and host logic -- C-ABI exports, GGUF contract, tokenizer,
prompt, size formulas, synthetic data.  No device calls."""
import os
import re

import numpy as np
import pytest

import oracle_py as op
import qasr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capi_exports_every_declared_symbol(built):
    hdr = open(os.path.join(ROOT, "include", "qasr_capi.h")).read()
    decl = set(re.findall(r"\b(qasr_[a-z0-9_]+)\s*\(", hdr))
    assert len(decl) >= 30
    lib = qasr.lib()
    missing = [n for n in sorted(decl) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(qasr.EXPORTS) <= decl
    assert qasr.lib().qasr_version().startswith(b"qasr-mi355x")


def test_size_formulas_match_reference(tiny_oracle):
    for n in [0, 1, 159, 160, 161, 16000, 480000, 1472000]:
        assert qasr.mel_frames(n) == n // 160
    for T in [0, 1, 2, 99, 100, 101, 199, 200, 3000, 9200]:
        assert qasr.encoder_frames(T) == op.olib().qo_enc_frames(T)
    assert qasr.encoder_frames(3000) == 390 and qasr.encoder_frames(9200) == 1196
    assert qasr.lib().qasr_prompt_len(390) == 405


def test_prompt_matches_reference_template(tiny_gguf, tiny_oracle):
    m = qasr.Model(tiny_gguf, -1)   # host-only load: no GPU involved
    ids, pos = m.build_prompt(5)
    # src/qwen3_asr.cpp:170-209 with an empty system prompt
    exp = [151644, 8948, 198, 151645, 198, 151644, 872, 198, 151669] + [151676] * 5 + \
          [151670, 151645, 198, 151644, 77091, 198]
    assert ids.tolist() == exp and pos == 9
    assert np.array_equal(ids, tiny_oracle.prompt(5))


def test_gguf_contract_of_synthetic_model(tiny_gguf):
    """names/shapes/dtypes follow scripts/convert_hf_to_gguf.py:50-120, 254-311
    and the shape imposition of src/gguf_loader.cpp:130-190."""
    g = op.Gguf(tiny_gguf)
    kv = g.kv
    assert kv["general.architecture"] == "qwen3-asr"
    C, D, H = int(kv["audio.conv_channels"]), int(kv["audio.d_model"]), int(kv["qwen3-asr.embedding_length"])
    t = g.tensors
    assert t["audio.encoder.conv1.weight"][0] == 1 and t["audio.encoder.conv1.weight"][1] == [3, 3, 1, C]
    assert t["audio.encoder.conv2.weight"][1] == [3, 3, C, C]
    assert t["audio.encoder.conv_out.weight"][1] == [C * 16, D]
    assert t["audio.encoder.blk.0.attn_q.bias"][0] == 0
    assert t["token_embd.weight"][1] == [H, 151936]
    assert "output.weight" not in t     # tied LM head
    for i in range(int(kv["qwen3-asr.block_count"])):
        for n in ("attn_norm", "attn_q", "attn_k", "attn_v", "attn_output", "attn_q_norm", "attn_k_norm", "ffn_norm",
                  "ffn_gate", "ffn_up", "ffn_down"):
            assert f"blk.{i}.{n}.weight" in t
    assert len(kv["tokenizer.ggml.tokens"]) == 151936


def test_host_only_model_and_hparams(tiny_gguf):
    m = qasr.Model(tiny_gguf, -1)
    hp = m.hp
    assert (hp.enc_layers, hp.d_model, hp.conv_channels, hp.hidden_size, hp.n_heads, hp.n_kv_heads) == (2, 256, 96, 256, 4, 2)
    assert hp.eos_id == 151645 and hp.audio_pad_id == 151676 and hp.weight_type == 1
    assert m.device_bytes == 0
    with pytest.raises(qasr.QasrError, match="host-only"):
        qasr.Context(m, 1, 64)


def test_tokenizer_decode_rules(tiny_gguf):
    """src/text_decoder.cpp:985-1075: <|..|> and [PAD..] skipped, GPT-2 byte
    unmapping (id 0..255 are the byte symbols)."""
    m = qasr.Model(tiny_gguf, -1)
    assert m.detokenize([151644, 151669, 151676, 151645, 151800]) == ""
    # byte symbols: '!'..'~' map to themselves
    assert m.detokenize([ord("H") - 0x21, ord("i") - 0x21]) == "Hi"
    # a synthetic word token 'ab' (id 256 -> 'a', 258 -> 'b'... ) round-trips through encode
    ids = m.tokenize("ab ab")
    assert m.detokenize(ids) == "ab ab"
    assert m.tokenize("") == []


def test_gguf_errors(tmp_path, built):
    p = tmp_path / "bad.gguf"
    p.write_bytes(b"GGUF\x03\x00\x00\x00" + b"\xff" * 16)
    with pytest.raises(qasr.QasrError):
        qasr.Model(str(p), -1)
    with pytest.raises(qasr.QasrError, match="open"):
        qasr.Model(str(tmp_path / "missing.gguf"), -1)


def test_synth_pcm_properties(built):
    a = qasr.synth_pcm(1000, 32000)
    assert np.array_equal(a, qasr.synth_pcm(1000, 32000))
    assert not np.array_equal(a, qasr.synth_pcm(1001, 32000))
    assert np.abs(a).max() <= 1.0 and 0.1 < a.std() < 0.4
    assert np.array_equal(np.round(a * 32768), a * 32768)     # PCM16-quantised like load_wav output


def test_wav_roundtrip(tmp_path, built):
    a = qasr.synth_pcm(42, 8000)
    p = str(tmp_path / "x.wav")
    qasr.write_wav(p, a)
    b, sr = qasr.load_wav(p)
    assert sr == 16000 and np.array_equal(a, b)


def test_stream_fetch_guard_stores_exception():
    """qasr._guarded_fetch: an exception in the Python fetch becomes -1 (queue
    empty) and is kept for the caller; later calls return -1 without calling
    fetch again"""
    import qasr
    failed, n = [], []

    def fetch(*a):
        n.append(1)
        raise KeyError("x")
    f = qasr._guarded_fetch(fetch, failed)
    assert f(None, None) == -1 and f(None, None) == -1
    assert len(n) == 1 and isinstance(failed[0], KeyError)
    ok = qasr._guarded_fetch(lambda *a: 7, [])
    assert ok(None) == 7


def test_ctx_grow_shape_bounds_kv_cells(built):
    """ADVICE r5 (Qwen3ASR::ensure_ctx): a context is recreated with the union
    of the old and the requested shape only while that union's KV cells do not
    exceed the larger of the two shapes -- 128 stream slots followed by a long
    single clip (16k positions) gives (1, 16k), not (128, 16k) (~240 GB of KV)"""
    import ctypes as C

    def grow(cb, cl, b, n):
        nb, nl = C.c_int(0), C.c_int(0)
        qasr.lib().qasr_ctx_grow_shape(cb, cl, b, n, C.byref(nb), C.byref(nl))
        return nb.value, nl.value
    assert grow(128, 600, 1, 16000) == (1, 16000)
    assert grow(1, 16000, 128, 600) == (128, 600)
    assert grow(0, 0, 4, 512) == (4, 512)
    assert grow(4, 512, 4, 600) == (4, 600)          # longer context, same slots: union
    assert grow(4, 512, 8, 512) == (8, 512)
    assert grow(64, 500, 128, 480) == (128, 480)     # union 64k cells > max(32k, 61.4k): the request alone
    assert grow(128, 480, 64, 500) == (64, 500)
