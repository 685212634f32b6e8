"""Known-answer tests of the reference's own test executables, on the real
Qwen3-ASR-0.6B GGUF (converted by the reference's scripts/convert_hf_to_gguf.py).
No weights exist offline, so every test here skips unless $QASR_MODEL names
that file; on a box that has it, they pin the whole path to the reference's
published answers:

  text-only "The capital of France is" -> 12095   tests/test_decoder_simple.cpp:36,72-76
  [audio_start, pad x3, audio_end]     -> 198     tests/test_decoder_last_pos.cpp:20,65-66
  audio_start + 48 pads + audio_end    -> 659     tests/test_decoder_50.cpp:54-55
  405-token chat prompt, no audio      -> 11528   tests/test_decoder_no_audio.cpp:21-51,86
  conv1 bias[0] = -0.062256, kernel[0,0] rows     tests/test_kernel_load.cpp:46-62
"""
import os

import numpy as np
import pytest

import oracle_py as op

MODEL = os.environ.get("QASR_MODEL", "")
pytestmark = pytest.mark.skipif(not os.path.isfile(MODEL), reason="$QASR_MODEL (real Qwen3-ASR-0.6B GGUF) not present")

IM_START, IM_END, SYS, USER, ASST, NL = 151644, 151645, 8948, 872, 77091, 198
A_START, A_PAD, A_END = 151669, 151676, 151670


def no_audio_prompt(n_pads=390):
    return ([IM_START, SYS, NL, IM_END, NL, IM_START, USER, NL, A_START] + [A_PAD] * n_pads +
            [A_END, IM_END, NL, IM_START, ASST, NL])


KATS = [
    ("france", [785, 6722, 315, 9625, 374], 12095),
    ("last_pos", [A_START, A_PAD, A_PAD, A_PAD, A_END], 198),
    ("pads50", [A_START] + [A_PAD] * 48 + [A_END], 659),
    ("no_audio", no_audio_prompt(), 11528),
]


def test_kat_conv1_weights():
    g = op.Gguf(MODEL)
    ty, ne, b = g.tensors["audio.encoder.conv1.bias"]
    assert ty == 0 and abs(float(b[0]) - (-0.062256)) < 5e-6
    ty, ne, w = g.tensors["audio.encoder.conv1.weight"]
    k = (w.astype(np.float32) if ty == 0 else w.view(np.float16).astype(np.float32))[:9].reshape(3, 3)
    want = np.array([[-0.003433, -0.037109, -0.117676], [-0.039062, -0.018311, 0.367188],
                     [0.005127, -0.037842, -0.218750]], np.float32)
    assert np.abs(k - want).max() < 2e-4   # printed to 6 places; an f16 file rounds them


@pytest.mark.parametrize("name,tokens,want", KATS, ids=[k[0] for k in KATS])
def test_kat_oracle(name, tokens, want):
    om = op.OracleModel(MODEL)
    lo = op.OracleDecoder(om, len(tokens) + 8).forward(np.asarray(tokens, np.int32), 0)
    assert int(np.argmax(lo)) == want


@pytest.mark.gpu
@pytest.mark.parametrize("name,tokens,want", KATS, ids=[k[0] for k in KATS])
def test_kat_gpu(gpu, name, tokens, want):
    import qasr
    m = qasr.Model(MODEL)
    c = qasr.Context(m, max_batch=1, max_ctx=len(tokens) + 8)
    try:
        _, am = c.prefill([np.asarray(tokens, np.int32)])
        assert int(am[0]) == want
    finally:
        c.close()
        m.close()
