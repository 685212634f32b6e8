"""CPU: the Q8_0 model format and the oracle's Q8_0 numerics.

The Q8_0 file follows scripts/convert_hf_to_gguf.py:230-308 (linear 2-D
weights Q8_0; conv kernels, token_embd, norms, biases F16/F32).  The oracle's
mul_mat restates ggml's Q8_0 x Q8_0 dot (activations quantised per 32 values).
Parity of these numerics to ggml itself is unpinned (no ggml in the reference
snapshot); these tests pin the block format and bound the quantisation error
against the F16 model generated from the same seed."""
import numpy as np

import oracle_py as op
import qasr

SR = 16000


def test_q8_file_follows_converter_policy(tiny_q8_gguf):
    g = op.Gguf(tiny_q8_gguf)
    t = g.tensors
    assert t["blk.0.attn_q.weight"][0] == 8 and t["blk.1.ffn_down.weight"][0] == 8
    assert t["audio.encoder.conv_out.weight"][0] == 8 and t["audio.encoder.proj2.weight"][0] == 8
    assert t["audio.encoder.blk.0.ffn_up.weight"][0] == 8
    for n in ("audio.encoder.conv1.weight", "audio.encoder.conv2.weight", "token_embd.weight"):
        assert t[n][0] == 1, n                     # conv last dim 3 / embeddings stay F16
    assert t["blk.0.attn_norm.weight"][0] == 0 and t["audio.encoder.blk.0.attn_q.bias"][0] == 0
    m = qasr.Model(tiny_q8_gguf, -1)
    assert m.hp.weight_type == 8


def test_q8_blocks_decode_to_f16_weights(tiny_gguf, tiny_q8_gguf):
    """block_q8_0 = fp16 d + 32 int8; d*q reproduces the F16 weight within half a quantum."""
    f = op.Gguf(tiny_gguf).tensors["blk.0.attn_k.weight"]
    q = op.Gguf(tiny_q8_gguf).tensors["blk.0.attn_k.weight"]
    w = f[2].view(np.float16).astype(np.float32).reshape(-1, 32)
    blk = np.asarray(q[2]).reshape(-1, 34)
    d = blk[:, :2].copy().view(np.float16).astype(np.float32)
    qs = blk[:, 2:].copy().view(np.int8).astype(np.float32)
    deq = d * qs
    amax = np.abs(w).max(axis=1, keepdims=True)
    assert np.all(np.abs(deq - w) <= amax / 127 * 0.5 + amax * 2e-3 + 1e-6)
    assert np.all(np.abs(qs).max(axis=1) == 127)


def test_oracle_q8_encoder_close_to_f16(tiny_oracle, tiny_q8_oracle):
    mel = op.log_mel(qasr.synth_pcm(4100, 2 * SR))
    a = tiny_oracle.encode_conv(mel)
    b = tiny_q8_oracle.encode_conv(mel)
    rel = np.abs(a - b).max() / np.abs(a).max()
    assert 0 < rel < 0.01, rel                     # int8 weights + int8 activations (measured 2e-3)
    a = tiny_oracle.encode(mel)
    b = tiny_q8_oracle.encode(mel)
    rel = np.abs(a - b).max() / np.abs(a).max()
    assert 0 < rel < 0.08, rel                     # measured 2.5e-2 after 2 layers + proj


def test_oracle_q8_decoder_runs(tiny_q8_oracle):
    pcm = qasr.synth_pcm(4200, SR)
    toks, _ = tiny_q8_oracle.transcribe(pcm, max_tokens=6, ignore_eos=True)
    assert len(toks) == 6 and all(0 <= t < 151936 for t in toks)
