"""CPU: forced-aligner host logic (src/forced_aligner.cpp) and its oracle --
GGUF contract of aligner files, hparams detection, tokenization with
timestamps, Korean split, pad count, LIS repair, CLI flag rules, and the
oracle's aligner encoder (padded chunks, 104-frame windows).  No device calls.

Parity note: the reference aligner needs ggml (absent), so these restate its
host functions in Python straight from src/forced_aligner.cpp and check the
product (C-ABI) and the C oracle against them."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as op
import qasr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "qwen3-asr.cpp_amd", "qwen3-asr-cli")
TS = 151705


@pytest.fixture(scope="session")
def al_tiny(built, tmp_path_factory):
    p = str(tmp_path_factory.mktemp("al") / "aligner-tiny.gguf")
    qasr.write_synthetic_gguf(p, "aligner-tiny", 42, 1)
    return p


@pytest.fixture(scope="session")
def al_oracle(al_tiny):
    op.set_threads(min(8, os.cpu_count() or 1))
    return op.OracleModel(al_tiny)


# --------------------------------------------------- restatements (Python)
def py_fix(data):
    """src/forced_aligner.cpp:1183-1265"""
    n = len(data)
    if n == 0:
        return []
    dp, parent = [1] * n, [-1] * n
    for i in range(1, n):
        for j in range(i):
            if data[j] <= data[i] and dp[j] + 1 > dp[i]:
                dp[i], parent[i] = dp[j] + 1, j
    mx, mi = 0, 0
    for i in range(n):
        if dp[i] > mx:
            mx, mi = dp[i], i
    normal = [False] * n
    i = mi
    while i != -1:
        normal[i] = True
        i = parent[i]
    r = list(data)
    i = 0
    while i < n:
        if normal[i]:
            i += 1
            continue
        j = i
        while j < n and not normal[j]:
            j += 1
        cnt = j - i
        lv = next((r[k] for k in range(i - 1, -1, -1) if normal[k]), -1)
        rv = next((r[k] for k in range(j, n) if normal[k]), -1)
        if cnt <= 2:
            for k in range(i, j):
                r[k] = rv if lv < 0 else (lv if rv < 0 else (lv if (k - (i - 1)) <= (j - k) else rv))
        elif lv >= 0 and rv >= 0:
            step = np.float32(rv - lv) / np.float32(cnt + 1)
            for k in range(i, j):
                r[k] = int(np.float32(lv) + step * np.float32(k - i + 1))
        elif lv >= 0:
            r[i:j] = [lv] * cnt
        elif rv >= 0:
            r[i:j] = [rv] * cnt
        i = j
    return r


def py_pads(T):
    """HF _get_feat_extract_output_lengths with C integer division (:1173-1178)"""
    leave = T % 100
    feat = int((leave - 1) / 2) + 1
    return int((int((feat - 1) / 2) + 1 - 1) / 2) + 1 + (T // 100) * 13


def py_korean(text, dic):
    """LTokenizer-style split (:1485-1541)"""
    out = []
    for w in text.split():
        if len(w) <= 2:
            out.append(w)
            continue
        best, be, bl, br = -1e9, 0, "", ""
        for e in range(2, len(w) + 1):
            sc = 1.0 if w[:e] in dic else 0.0
            if sc > best or (sc == best and e > be):
                best, be, bl, br = sc, e, w[:e], w[e:]
        out.append(bl)
        if br:
            out.append(br)
    return out


# ------------------------------------------------------------------ tests
def test_aligner_gguf_contract_and_hparams(al_tiny, built, tmp_path):
    g = op.Gguf(al_tiny)
    kv, t = g.kv, g.tensors
    assert kv["qwen3-asr.classify_num"] == 5000 and kv["qwen3-asr.timestamp_token_id"] == TS
    assert kv["qwen3-asr.timestamp_segment_time"] == 80
    H = int(kv["qwen3-asr.embedding_length"])
    assert t["output.weight"][0] == 1 and t["output.weight"][1] == [H, 5000]
    assert kv["tokenizer.ggml.tokens"][TS] == "<timestamp>"
    m = qasr.Model(al_tiny, -1)
    assert m.is_aligner and m.hp.classify_num == 5000 and m.hp.timestamp_token_id == TS
    assert (m.hp.enc_layers, m.hp.d_model) == (2, 256)
    # Q8_0 aligner: the classify head stays F16 (convert_hf_to_gguf.py:240-241)
    q = str(tmp_path / "al-q8.gguf")
    qasr.write_synthetic_gguf(q, "aligner-tiny", 42, 8)
    gq = op.Gguf(q)
    assert gq.tensors["output.weight"][0] == 1 and gq.tensors["blk.0.attn_q.weight"][0] == 8
    # an ASR file is not an aligner
    a = str(tmp_path / "asr.gguf")
    qasr.write_synthetic_gguf(a, "tiny", 42, 1)
    assert not qasr.Model(a, -1).is_aligner


@pytest.mark.parametrize("data", [[], [3], [5, 3, 8, 9, 2, 10], [0, 0, 0], [9, 8, 7, 6, 5], [1, 50, 2, 3, 4, 60, 5, 6],
                                  [10, 11, 12, 3, 4, 5, 13, 14], [100, 1, 2, 3, 4, 5, 6, 7], [4, 4, 2, 2, 9, 9, 1, 1]])
def test_fix_timestamps_matches_restatement(data, built):
    assert qasr.fix_timestamps(data) == py_fix(data)


def test_fix_timestamps_random_monotone(built):
    rng = np.random.default_rng(0)
    for n in [1, 2, 7, 40, 200]:
        d = np.sort(rng.integers(0, 400, n)).tolist()
        for _ in range(n // 5 + 1):   # a few outliers
            d[int(rng.integers(0, n))] = int(rng.integers(0, 400))
        r = qasr.fix_timestamps(d)
        assert r == py_fix(d)


@pytest.mark.parametrize("T", [1, 2, 99, 100, 101, 199, 200, 250, 3000, 9200, 9201])
def test_pad_count_formula(T, built):
    n = T * 160 + 37
    assert qasr.align_prompt_len(n, 7) == 7 + 2 + py_pads(T)
    # equals the encoder's own frame count except at whole chunks (+1 there)
    assert py_pads(T) == qasr.encoder_frames(T) + (1 if T % 100 == 0 else 0)


def test_tokenize_with_timestamps(al_tiny):
    m = qasr.Model(al_tiny, -1)
    text = "  ab  cd\tef\nab "
    ids, nw = m.align_tokenize(text)
    assert nw == 4 and m.align_words(text) == ["ab", "cd", "ef", "ab"]
    exp = []
    for w in ["ab", "cd", "ef", "ab"]:   # no leading-space marker on any word (:1592)
        exp += m.tokenize(w) + [TS, TS]
    assert ids == exp
    assert m.align_tokenize("") == ([], 0)


def test_korean_split(al_tiny, tmp_path):
    m = qasr.Model(al_tiny, -1)
    words = ["안녕", "하세요", "세계"]
    d = tmp_path / "dict.txt"
    d.write_text("안녕하 3 n\n세계 9\n\n하세 1\n", encoding="utf-8")
    m.load_korean_dict(str(d))
    dic = {"안녕하", "세계", "하세"}
    for text in ["안녕하세요 세계", "하세요요 가", "세계평화 안녕", "가나다라"]:
        assert m.align_words(text, "korean") == py_korean(text, dic), text
        # non-Korean language: whitespace split only
        assert m.align_words(text) == text.split()
    with pytest.raises(qasr.QasrError):
        m.load_korean_dict(str(tmp_path / "missing.dict"))
    del words


def test_oracle_aligner_encoder_padding_and_windows(al_oracle):
    """chunks zero-padded to 100 frames (the short last chunk differs from the
    ASR's unpadded one) and attention confined to 104-frame windows: mel past
    frame 800 (= 8 chunks = 104 encoder frames) cannot move the first window."""
    rng = np.random.default_rng(5)
    mel = op.log_mel(qasr.synth_pcm(77, 16000 * 11 + 3210))   # 1120 frames -> 2 windows
    T = mel.shape[1]
    a = al_oracle.encode(mel)
    assert a.shape == (qasr.encoder_frames(T), al_oracle.m.hidden)
    mel2 = mel.copy()
    mel2[:, 800:] += rng.standard_normal((128, T - 800)).astype(np.float32)
    b = al_oracle.encode(mel2)
    assert np.array_equal(a[:104], b[:104])
    assert not np.array_equal(a[104:], b[104:])
    # padded vs unpadded last chunk: conv outputs of the last valid frames differ
    c = al_oracle.encode_conv(mel[:, :150])
    al_oracle.m.aligner = 0
    try:
        d = al_oracle.encode_conv(mel[:, :150])
    finally:
        al_oracle.m.aligner = 1
    assert c.shape == d.shape == (13 + 7, al_oracle.m.d_model)
    assert np.array_equal(c[:13], d[:13]) and not np.array_equal(c[13:], d[13:])


def test_oracle_align_classes_shape(al_oracle, al_tiny):
    m = qasr.Model(al_tiny, -1)
    ids, nw = m.align_tokenize("ab cd ef")
    cls, lg, toks = al_oracle.align_classes(qasr.synth_pcm(9, 16000 * 2), ids)
    assert len(cls) == 2 * nw == 6 and lg.shape == (6, 5000)
    assert toks[0] == 151669 and toks[1:1 + py_pads(200)] == [151676] * py_pads(200)
    assert all(0 <= c < 5000 for c in cls)


def test_cli_alignment_flag_rules(built):
    def run(*a):
        return subprocess.run([CLI, *a], capture_output=True, text=True)
    r = run("-m", "x.gguf", "-f", "a.wav", "--align")
    assert r.returncode == 1 and "Reference text is required for alignment mode (--text)" in r.stderr
    r = run("-m", "x.gguf", "-f", "a.wav", "--align", "--text", "hi", "-a")
    assert r.returncode == 1 and "cannot be used together" in r.stderr
    r = run("-m", "x.gguf", "-f", "a.wav", "--transcribe-align")
    assert r.returncode == 1 and "--aligner-model is required" in r.stderr
    r = run("--help")
    assert r.returncode == 0 and "--transcribe-align" in r.stderr
