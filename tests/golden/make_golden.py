#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REFERENCE's own code.

Runs the reference's src/mel_spectrogram.cpp and src/audio_injection.cpp,
compiled in place by `make -C oracle ref` into oracle/_ref/libqasr_ref.so
(the only reference translation units that build without the absent ggml).
Inputs are the product's deterministic synthetic clips (qasr_synth_pcm),
whose bytes are pinned here by SHA-256 as well.  Outputs are data only
(inputs + expected outputs); no reference source is stored.

    python tests/golden/make_golden.py
"""
import hashlib
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))

import ctypes as C  # noqa: E402

import oracle_py as op  # noqa: E402
import qasr  # noqa: E402

# (seed, n_samples): 1 s, 2.5 s, 7.3 s (odd length), edge lengths, 30 s
SMALL = [(1000, 16000), (1001, 40000), (1002, 116800), (1003, 0), (1004, 159), (1005, 160), (1006, 401), (1008, 16123)]
LARGE = [(1007, 480000)]
SUB = 97   # subsampling stride for the 30 s mel


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def wav_bytes(samples_i16: np.ndarray, channels: int, sr: int) -> bytes:
    data = samples_i16.astype("<i2").tobytes()
    fmt = struct.pack("<HHIIHH", 1, channels, sr, sr * channels * 2, channels * 2, 16)
    extra = b"LIST" + struct.pack("<I", 4) + b"INFO"          # an unknown chunk the reader must skip
    body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + extra + b"data" + struct.pack("<I", len(data)) + data
    return b"RIFF" + struct.pack("<I", len(body)) + body


def main():
    if not op.have_ref():
        raise SystemExit("oracle/_ref/libqasr_ref.so missing: run `make -C oracle ref` (needs /root/reference)")
    out = {}
    out["filters"] = op.ref_mel_filters()
    for seed, n in SMALL:
        pcm = qasr.synth_pcm(seed, n)
        out[f"pcm_sha_{seed}"] = np.array(sha(pcm))
        out[f"mel_{seed}"] = op.ref_log_mel(pcm)
    for seed, n in LARGE:
        pcm = qasr.synth_pcm(seed, n)
        mel = op.ref_log_mel(pcm)
        out[f"pcm_sha_{seed}"] = np.array(sha(pcm))
        out[f"mel_sha_{seed}"] = np.array(sha(mel))
        out[f"mel_shape_{seed}"] = np.array(mel.shape)
        out[f"mel_sub_{seed}"] = mel.ravel()[::SUB].copy()
        out[f"mel_colsum_{seed}"] = mel.astype(np.float64).sum(axis=0)
    # reference audio_injection semantics on the reference test's own inputs
    # (tests/test_injection.cpp: ids {151669, 151676 x3, 151670}, vocab 10 x 4 table)
    V, Hd = 200000, 8
    table = (np.arange(V, dtype=np.float32)[:, None] % 1000 + np.arange(Hd, dtype=np.float32)[None, :] / 10000).astype(np.float32)
    ids = np.array([151669, 151676, 151676, 151676, 151670], np.int32)
    audio = (500 + np.arange(3, dtype=np.float32)[:, None] + np.arange(Hd, dtype=np.float32)[None, :] / 10000).astype(np.float32)
    emb = np.zeros((5, Hd), np.float32)
    rc = op.rlib().ref_inject_audio(ids.ctypes.data_as(C.POINTER(C.c_int32)), 5, op._f(audio), 3, op._f(table), V, Hd, 151676,
                                    op._f(emb))
    assert rc == 5
    out["inject_ids"] = ids
    out["inject_audio"] = audio
    out["inject_expected"] = emb
    # WAV reader: stereo PCM16 with an extra chunk -> channel mean / 32768
    rng = np.random.default_rng(5)
    st = rng.integers(-32768, 32767, size=(257, 2)).astype(np.int16)
    wb = wav_bytes(st.ravel(), 2, 16000)
    path = os.path.join(HERE, "_tmp_stereo.wav")
    with open(path, "wb") as f:
        f.write(wb)
    n = op.rlib().ref_load_wav(path.encode(), None, 0, None)
    ref_s = np.zeros(n, np.float32)
    srv = C.c_int(0)
    op.rlib().ref_load_wav(path.encode(), op._f(ref_s), n, C.byref(srv))
    os.remove(path)
    out["wav_bytes"] = np.frombuffer(wb, np.uint8)
    out["wav_expected"] = ref_s
    out["wav_sr"] = np.array(srv.value)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print("wrote", os.path.join(HERE, "golden.npz"), sorted(out.keys()))


if __name__ == "__main__":
    main()
