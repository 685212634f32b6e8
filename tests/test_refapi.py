"""The reference's own driver programs against this repo's component API.

tools/refapi/Makefile compiles 17 of the reference's tests/*.cpp -- every one
that includes only the component headers (mel_spectrogram.h, audio_encoder.h,
text_decoder.h, audio_injection.h) -- in place and unchanged, against
include/ + libqasr.so, in the build container.  Here:

* (CPU) every one of them compiled and linked, and test_injection.cpp (host
  code only) passes its own checks;
* (GPU) test_mel.cpp and test_encoder.cpp run their own comparisons on
  synthetic inputs whose expected outputs come from the oracle (mel:
  bit-exact to the reference's mel_spectrogram.cpp, tests/test_oracle_golden.py;
  encoder: the restated ggml numerics), at the drivers' own tolerances (mel
  1e-5, encoder 2e-2 max |delta|); test_decoder_last_pos.cpp
  runs the TextDecoder on the synthetic full-size GGUF: its printed argmax
  of the one row of logits forward returns equals the C-ABI prefill's
  (test_decoder_no_audio.cpp reads 404 rows past that row, on the reference
  too: compiled only).
Random-init weights: the drivers' known answers (12095, 198, 11528) are
real-weight facts (tests/test_kat_real_weights.py) and are not asserted.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_py as op
import qasr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "refapi", "_out")
REF = "/root/reference/tests"
DRIVERS = ["test_decoder_simple", "test_decoder_last_pos", "test_decoder_no_audio", "test_encoder",
           "test_attention_compare", "test_conv_no_chunk", "test_conv_only", "test_decoder", "test_decoder_50",
           "test_decoder_debug", "test_decoder_lengths", "test_decoder_trace", "test_decoder_with_audio",
           "test_encoder_no_chunk", "test_injection", "test_mel", "test_qk_compare"]
SR = 16000


def _npy(path, a):
    np.save(path, np.ascontiguousarray(a, dtype=np.float32))


def _run(args, cwd, timeout=240):
    env = dict(os.environ)
    return subprocess.run(args, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference sources exist only in the build container")
def test_reference_drivers_compile_against_component_api():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tools", "refapi")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for d in DRIVERS:
        assert os.path.isfile(os.path.join(OUT, d)), d


def test_reference_injection_driver(tmp_path):
    """src/audio_injection.h's helpers: the reference's test_injection.cpp, host only"""
    exe = _need("test_injection")
    r = _run([exe], str(tmp_path))
    assert r.returncode == 0 and "All tests passed" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def _need(name):
    """the driver binary: __graft_entry__.build() compiles them in the build
    container (where /root/reference exists) and they travel with the tree,
    so a missing one is a failure, not a skip"""
    exe = os.path.join(OUT, name)
    if not os.path.isfile(exe):
        pytest.fail(f"tools/refapi/_out/{name} missing: run __graft_entry__.build() (make -C tools/refapi) in the "
                    "build container before the GPU run")
    return exe


@pytest.mark.gpu
def test_reference_mel_driver(gpu, tmp_path):
    """test_mel.cpp: load_wav + load_mel_filters_npy + log_mel_spectrogram
    (our GPU mel) against a reference mel .npy, its own 1e-5 tolerance"""
    exe = _need("test_mel")
    pcm = qasr.synth_pcm(4242, int(4.3 * SR))
    wav = tmp_path / "sample.wav"
    qasr.write_wav(str(wav), pcm)
    pcm16 = np.asarray(qasr.load_wav(str(wav))[0], np.float32)   # what the driver reads back
    mel = op.log_mel(pcm16)
    os.makedirs(tmp_path / "tests" / "reference")
    _npy(tmp_path / "tests" / "reference" / "mel.npy", mel)
    filt = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))["filters"]   # [128][201]
    _npy(tmp_path / "tests" / "reference" / "mel_filters.npy", filt.T)             # the file layout (201, 128)
    r = _run([exe, "--audio", str(wav)], str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    got = np.load(tmp_path / "tests" / "output" / "mel_computed.npy")
    assert got.shape == mel.shape and float(np.abs(got - mel).max()) <= 1e-5


@pytest.mark.gpu
def test_reference_encoder_driver(gpu, tiny_gguf, tiny_oracle, tmp_path):
    """test_encoder.cpp: AudioEncoder::load_model + encode against the oracle's
    features, the driver's own 2e-2 max |delta| bar"""
    exe = _need("test_encoder")
    mel = op.log_mel(qasr.synth_pcm(4343, int(3.7 * SR)))
    feats = tiny_oracle.encode(mel)
    _npy(tmp_path / "mel.npy", mel)
    _npy(tmp_path / "feats.npy", feats)
    r = _run([exe, "--model", tiny_gguf, "--mel", str(tmp_path / "mel.npy"), "--ref", str(tmp_path / "feats.npy")], str(tmp_path))
    assert r.returncode == 0 and "TEST PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_reference_decoder_driver_last_pos(gpu, full_f16_gguf, tmp_path):
    """TextDecoder::load_model / init_kv_cache / forward on the synthetic
    full-size model (test_decoder_last_pos.cpp).  forward returns the last
    row's logits only, as the reference's graph does (src/text_decoder.cpp:
    563-565 views row n_tokens-1 before the norm; :674-677 copies ne[1] = 1
    row).  The driver still indexes logits + (n_tokens - 1) * vocab_size --
    past the end of that vector on the reference too -- so its "LAST
    position" lines are undefined and not read; its "Position 0 argmax"
    (row 0 = the one row returned) must equal the C-ABI prefill's argmax.
    test_decoder_no_audio.cpp makes the same read 404 rows past the end (a
    segfault on the reference as here), so it is compiled, not run."""
    exe = _need("test_decoder_last_pos")
    os.makedirs(tmp_path / "models")
    os.symlink(full_f16_gguf, tmp_path / "models" / "qwen3-asr-0.6b-f16.gguf")
    r = _run([exe], str(tmp_path), timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    top = re.search(r"Position 0 argmax: (\d+) \(logit=([-0-9.]+)\)", r.stdout)
    assert top, r.stdout[-2000:]
    ids = [151669] + [151676] * 3 + [151670]
    m = qasr.Model(full_f16_gguf)
    c = qasr.Context(m, max_batch=1, max_ctx=len(ids) + 8)
    try:
        lg, am = c.prefill([ids])
    finally:
        c.close()
        m.close()
    assert int(top.group(1)) == int(am[0])
    assert abs(float(top.group(2)) - float(lg[0][int(am[0])])) <= 1e-3 * max(1.0, abs(float(top.group(2))))


@pytest.mark.gpu
def test_reference_encoder_no_chunk_driver(gpu, full_f16_gguf, tmp_path):
    """test_encoder_no_chunk.cpp unchanged: AudioEncoder::encode_no_chunk on the
    full-size model (its hard-coded models/qwen3-asr-0.6b-f16.gguf, here the
    synthetic one) against tests/reference/encoder_no_chunk.npy, which the
    oracle's QO_ENC_NO_CHUNK writes; the driver's own 2e-2 max |delta| bar"""
    exe = _need("test_encoder_no_chunk")
    om = op.OracleModel(full_f16_gguf)
    mel = op.log_mel(qasr.synth_pcm(4344, int(2.6 * SR)))   # 260 frames: three chunks in encode()
    (tmp_path / "tests" / "reference").mkdir(parents=True)
    (tmp_path / "models").mkdir()
    os.symlink(full_f16_gguf, tmp_path / "models" / "qwen3-asr-0.6b-f16.gguf")
    _npy(tmp_path / "tests" / "reference" / "mel.npy", mel)
    _npy(tmp_path / "tests" / "reference" / "encoder_no_chunk.npy", om.encode(mel, op.OracleModel.ENC_NO_CHUNK))
    r = _run([exe], str(tmp_path))
    assert r.returncode == 0 and "TEST PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
