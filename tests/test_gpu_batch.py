"""GPU: the decode-batch kernels (B > 8: gemm_skinny_kernel / gemm_skinny_q8_kernel
row blocks and K-split waves, the attention -- one workgroup per (kv group,
sequence) streaming that sequence's keys (decode_attn_seq_kernel) once the
batch fills the CUs, 256-key splits below that --, the skinny LM head with
argmax, Q8_0 quantisation fused into the norm and the attention combiner) at
the batch sizes the bench runs.

Every row of a batch holds the same sequence, so every row must come out
bit-identical to row 0 (an output row depends only on its own inputs and on
the same instruction sequence, whatever row block or tile it lands in), and
row 0 must match the oracle within the tolerances of tests/test_gpu_parity.py
(F16) and tests/test_gpu_q8.py (Q8_0; both against the default oracle: the decode
attention accumulates V.P in fp16 as ggml's CPU flash attention)."""
import numpy as np
import pytest

import oracle_py as op
import qasr

pytestmark = pytest.mark.gpu
SR = 16000


@pytest.mark.parametrize("B,secs", [(64, 1.3), (100, 1.3), (64, 24.0)])
@pytest.mark.parametrize("path", ["f16", "q8"])
def test_decode_batch_rows_identical_and_match_oracle(path, B, secs, gpu, tiny_gguf, tiny_q8_gguf, tiny_oracle,
                                                      tiny_q8_oracle):
    """(64, 24 s): a ~330-token context, so the 256-key attention splits and
    their combine run with more than one split per sequence"""
    q8 = path == "q8"
    om = tiny_q8_oracle if q8 else tiny_oracle
    m = qasr.Model(tiny_q8_gguf if q8 else tiny_gguf)
    feats = om.encode(op.log_mel(qasr.synth_pcm(9100 + B, int(secs * SR))))
    ids, pos = m.build_prompt(feats.shape[0])
    steps = 3
    c = qasr.Context(m, max_batch=B, max_ctx=len(ids) + steps + 8)
    try:
        _, am = c.prefill([ids] * B, [feats] * B, [pos] * B, want_logits=False)
        assert len(set(int(a) for a in am)) == 1
        tok0 = int(am[0])
        toks, out = [tok0] * B, []
        for s in range(steps):
            lg, am = c.decode_step(toks, [len(ids) + s] * B)
            out.append(lg)
            toks = [int(am[0])] * B
    finally:
        c.close()
        m.close()
    for s, lg in enumerate(out):
        for b in range(1, B):
            assert np.array_equal(lg[b], lg[0]), (s, b)
    dec = op.OracleDecoder(om, len(ids) + steps + 8)
    dec.forward(ids, 0, feats, pos)
    ref = dec.forward([tok0], len(ids))   # the first decode step, same fed token
    scale = float(np.abs(ref).max())
    tol = (2e-2 if q8 else 1e-2) * scale
    assert np.abs(out[0][0] - ref).max() <= tol, (np.abs(out[0][0] - ref).max(), tol)


@pytest.mark.parametrize("B", [1, 3])
def test_decode_long_context_splits(B, gpu, tiny_gguf, tiny_oracle):
    """contexts past 1k keys: batch <= 8 switches to 128-key attention splits
    (13 of them here); text-only prompt of 1100 ids, every row against the oracle"""
    m = qasr.Model(tiny_gguf)
    rng = np.random.default_rng(21)
    ids = [int(t) for t in rng.integers(0, 151643, 1100)]
    c = qasr.Context(m, max_batch=B, max_ctx=1200)
    try:
        c.prefill([ids] * B, want_logits=False)
        toks = [int(t) for t in rng.integers(0, 151643, 3)]
        outs = []
        for s, t in enumerate(toks):
            lg, _ = c.decode_step([t] * B, [len(ids) + s] * B)
            outs.append(lg)
    finally:
        c.close()
        m.close()
    dec = op.OracleDecoder(tiny_oracle, 1200)
    dec.forward(ids, 0)
    for s, t in enumerate(toks):
        ref = dec.forward([t], len(ids) + s)
        tol = 1e-2 * float(np.abs(ref).max())
        for b in range(B):
            assert np.abs(outs[s][b] - ref).max() <= tol, (s, b, np.abs(outs[s][b] - ref).max(), tol)


@pytest.mark.parametrize("path", ["f16", "q8"])
def test_decode_batch_ragged_contexts(path, gpu, tiny_gguf, tiny_q8_gguf, tiny_oracle, tiny_q8_oracle):
    """a batch of 40 rows with two different prompts (2.1 s and 9.7 s clips,
    alternating): each sequence attends over its own context only (the
    per-sequence attention loads keys up to its own position); rows of the same
    clip bit-identical, row 0 / row 1 against the oracle"""
    q8 = path == "q8"
    om = tiny_q8_oracle if q8 else tiny_oracle
    m = qasr.Model(tiny_q8_gguf if q8 else tiny_gguf)
    B, steps = 40, 3
    fs = [om.encode(op.log_mel(qasr.synth_pcm(9300 + k, int(sec * SR)))) for k, sec in enumerate((2.1, 9.7))]
    pr = [m.build_prompt(f.shape[0]) for f in fs]
    c = qasr.Context(m, max_batch=B, max_ctx=max(len(p[0]) for p in pr) + steps + 8)
    try:
        _, am = c.prefill([pr[b % 2][0] for b in range(B)], [fs[b % 2] for b in range(B)], [pr[b % 2][1] for b in range(B)],
                          want_logits=False)
        tok0 = [int(am[0]), int(am[1])]
        toks, out = [tok0[b % 2] for b in range(B)], []
        for s in range(steps):
            lg, am = c.decode_step(toks, [len(pr[b % 2][0]) + s for b in range(B)])
            out.append(lg)
            toks = [int(am[b % 2]) for b in range(B)]
    finally:
        c.close()
        m.close()
    for lg in out:
        for b in range(2, B):
            assert np.array_equal(lg[b], lg[b % 2]), b
    for k in range(2):
        ids, pos = pr[k]
        dec = op.OracleDecoder(om, len(ids) + steps + 8)
        dec.forward(ids, 0, fs[k], pos)
        ref = dec.forward([tok0[k]], len(ids))
        tol = (2e-2 if q8 else 1e-2) * float(np.abs(ref).max())
        assert np.abs(out[0][k] - ref).max() <= tol, (k, np.abs(out[0][k] - ref).max(), tol)


@pytest.mark.parametrize("B", [1, 48])
def test_decode_kv_nt_bit_identical_and_attention_kernels_agree(B, gpu, tiny_gguf, tiny_oracle):
    """kv_nt (K/V cache rows loaded nontemporal, default on) reads the same
    bytes: bit-identical decode-step logits with it off.  At B = 48 also the
    split-K batch attention (att_stream = 0) against the per-sequence kernel:
    different merge order, so equal within the oracle tolerance, and both
    against the oracle.  Both are the fp32-accumulating attention (option
    fa_exact_decode = 0), so the oracle runs its QO_FA_V_F32 switch."""
    m = qasr.Model(tiny_gguf)
    rng = np.random.default_rng(9)
    ids = [int(t) for t in rng.integers(0, 151643, 300)]
    toks = [int(t) for t in rng.integers(0, 151643, 3)]
    runs = {}
    try:
        for cfg in ((1, 1), (0, 1), (1, 0)):
            if B == 1 and cfg[1] == 0:
                continue
            c = qasr.Context(m, max_batch=B, max_ctx=320)
            c.set_option("kv_nt", cfg[0])
            c.set_option("att_stream", cfg[1])
            c.set_option("fa_exact_decode", 0)
            try:
                c.prefill([ids] * B, want_logits=False)
                runs[cfg] = [c.decode_step([t] * B, [len(ids) + s] * B)[0].copy() for s, t in enumerate(toks)]
            finally:
                c.close()
    finally:
        m.close()
    for a, b in zip(runs[(1, 1)], runs[(0, 1)]):
        assert np.array_equal(a, b)
    dec = op.OracleDecoder(tiny_oracle, 320, op.OracleModel.FA_V_F32)
    dec.forward(ids, 0)
    for s, t in enumerate(toks):
        ref = dec.forward([t], len(ids) + s)
        tol = 1e-2 * float(np.abs(ref).max())
        for cfg, out in runs.items():
            assert np.abs(out[s][0] - ref).max() <= tol, (cfg, s)
