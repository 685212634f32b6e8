"""Python side of the CPU oracle (TEST INFRASTRUCTURE ONLY).

- an independent GGUF v3 reader (numpy memmap; not the product's C++ parser),
- ctypes bindings of oracle/liboracle.so (the C restatement of the reference
  path, oracle/qasr_oracle.c),
- bindings of oracle/_ref/libqasr_ref.so (the reference's own
  mel_spectrogram.cpp / audio_injection.cpp) when it has been built.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF_LIB = os.path.join(ORACLE_DIR, "_ref", "libqasr_ref.so")


# ------------------------------------------------------------------ GGUF read
GGUF_TYPES = {0: "u1", 1: "i1", 2: "<u2", 3: "<i2", 4: "<u4", 5: "<i4", 6: "<f4", 7: "u1", 10: "<u8", 11: "<i8", 12: "<f8"}


class Gguf:
    def __init__(self, path: str):
        self.path = path
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        buf = self.mm
        p = 0

        def rd(fmt):
            nonlocal p
            v = struct.unpack_from(fmt, buf, p)
            p += struct.calcsize(fmt)
            return v[0] if len(v) == 1 else v

        def rstr():
            nonlocal p
            n = rd("<Q")
            s = bytes(buf[p:p + n]).decode("utf-8", errors="surrogateescape")
            p += n
            return s

        def rval(t):
            nonlocal p
            if t == 8:
                return rstr()
            if t == 9:
                at, n = rd("<I"), rd("<Q")
                if at == 8:
                    return [rstr() for _ in range(n)]
                dt = np.dtype(GGUF_TYPES[at])
                a = np.frombuffer(buf, dt, n, p)
                p += n * dt.itemsize
                return a
            dt = np.dtype(GGUF_TYPES[t])
            v = np.frombuffer(buf, dt, 1, p)[0]
            p += dt.itemsize
            return v.item()

        magic, ver = rd("<I"), rd("<I")
        assert magic == 0x46554747, "bad GGUF magic"
        assert ver in (2, 3)
        nt, nkv = rd("<Q"), rd("<Q")
        self.kv = {}
        for _ in range(nkv):
            k = rstr()
            t = rd("<I")
            self.kv[k] = rval(t)
        self.tensors = {}
        infos = []
        for _ in range(nt):
            name = rstr()
            nd = rd("<I")
            ne = [rd("<Q") for _ in range(nd)]
            ty, off = rd("<I"), rd("<Q")
            infos.append((name, ne, ty, off))
        align = int(self.kv.get("general.alignment", 32))
        data = (p + align - 1) // align * align
        for name, ne, ty, off in infos:
            n = int(np.prod(ne))
            if ty == 0:
                arr = np.frombuffer(buf, np.float32, n, data + off)
            elif ty == 1:
                arr = np.frombuffer(buf, np.uint16, n, data + off)
            elif ty == 8:
                arr = np.frombuffer(buf, np.uint8, n // 32 * 34, data + off)
            else:
                raise ValueError(f"unsupported ggml type {ty} for {name}")
            self.tensors[name] = (ty, ne, arr)

    def t(self, name):
        return self.tensors[name][2]


# ------------------------------------------------------------------- oracle
def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


class EncLayer(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "attn_q_w", "attn_k_w", "attn_v_w", "attn_out_w", "attn_q_b", "attn_k_b", "attn_v_b", "attn_out_b",
        "attn_norm_w", "attn_norm_b", "ffn_up_w", "ffn_down_w", "ffn_up_b", "ffn_down_b", "ffn_norm_w", "ffn_norm_b")]


class DecLayer(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "attn_norm", "attn_q_norm", "attn_k_norm", "ffn_norm", "attn_q", "attn_k", "attn_v", "attn_output",
        "ffn_gate", "ffn_up", "ffn_down")]


class QoModel(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("enc_layers", "d_model", "enc_heads", "enc_ffn", "conv_ch", "n_mel")] + [
        ("enc_eps", C.c_float)] + [(n, C.c_int) for n in (
            "vocab", "hidden", "dec_layers", "n_head", "n_kv_head", "head_dim", "dec_ffn")] + [
        ("rms_eps", C.c_float), ("rope_theta", C.c_float)] + [(n, C.c_int) for n in (
            "eos_id", "audio_start_id", "audio_end_id", "audio_pad_id", "wtype")] + [(n, C.c_void_p) for n in (
        "conv1_w", "conv2_w", "conv3_w", "conv_out_w", "conv1_b", "conv2_b", "conv3_b", "ln_post_w", "ln_post_b",
        "proj1_w", "proj2_w", "proj1_b", "proj2_b")] + [("enc", C.POINTER(EncLayer)), ("token_embd", C.c_void_p),
                                                        ("output_norm", C.c_void_p), ("dec", C.POINTER(DecLayer)),
                                                        ("aligner", C.c_int), ("classify_num", C.c_int),
                                                        ("classify_w", C.c_void_p)]


_olib = None


def olib():
    global _olib
    if _olib is None:
        if not os.path.exists(ORACLE_LIB):
            build_oracle()
        L = C.CDLL(ORACLE_LIB)
        F, I = C.POINTER(C.c_float), C.c_int
        L.qo_mel_filters.argtypes = [F]
        L.qo_log_mel.argtypes = [F, I, F, F]
        L.qo_log_mel.restype = I
        L.qo_load_wav.argtypes = [C.c_char_p, F, I, C.POINTER(I)]
        L.qo_enc_frames.argtypes = [I]
        L.qo_encode_conv.argtypes = [C.POINTER(QoModel), F, I, F, I]
        L.qo_encode.argtypes = [C.POINTER(QoModel), F, I, F, I]
        L.qo_dec_new.argtypes = [C.POINTER(QoModel), I, I]
        L.qo_dec_new.restype = C.c_void_p
        L.qo_dec_free.argtypes = [C.c_void_p]
        L.qo_dec_forward.argtypes = [C.c_void_p, C.POINTER(C.c_int32), I, F, I, I, I, F]
        L.qo_argmax.argtypes = [F, I]
        L.qo_argmax.restype = C.c_int32
        L.qo_build_prompt.argtypes = [C.POINTER(QoModel), I, C.POINTER(C.c_int32)]
        L.qo_transcribe.argtypes = [C.POINTER(QoModel), F, I, I, I, I, C.POINTER(C.c_int32), C.POINTER(C.c_double)]
        L.qo_set_threads.argtypes = [I]
        L.qo_align_forward.argtypes = [C.POINTER(QoModel), C.POINTER(C.c_int32), I, F, I, I, C.POINTER(I), I, F, I]
        L.qo_f32_to_f16.argtypes = [C.c_float]
        L.qo_f32_to_f16.restype = C.c_uint16
        for fn in (L.qo_f16_mad_round1, L.qo_f16_mad_round2):
            fn.argtypes = [C.c_uint16, C.c_float, C.c_uint16]
            fn.restype = C.c_uint16
        _olib = L
    return _olib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def set_threads(n: int) -> None:
    olib().qo_set_threads(n)


def mel_filters() -> np.ndarray:
    out = np.zeros(128 * 201, np.float32)
    olib().qo_mel_filters(_f(out))
    return out.reshape(128, 201)


def log_mel(pcm: np.ndarray) -> np.ndarray:
    pcm = np.ascontiguousarray(pcm, np.float32)
    fil = mel_filters().ravel().copy()
    T = olib().qo_log_mel(_f(pcm), len(pcm), _f(fil), None)
    out = np.zeros(max(1, 128 * T), np.float32)
    olib().qo_log_mel(_f(pcm), len(pcm), _f(fil), _f(out))
    return out[:128 * T].reshape(128, T)


class OracleModel:
    """qo_model view of a GGUF file (keeps the memmap alive)."""

    GELU_EXACT = 1
    FA_V_F32 = 2
    FA_V_ROUND1 = 4   # fp16 V accumulation with one rounding per key (qasr_oracle.h QO_FA_V_ROUND1)
    ENC_NO_CHUNK = 8  # AudioEncoder::encode_no_chunk: the conv stack over all frames, PE 0..N-1

    def __init__(self, path: str):
        g = Gguf(path)
        self.g = g
        kv = g.kv

        def k2(a, b, d):
            return int(kv[a]) if a in kv else int(kv.get(b, d))

        m = QoModel()
        # ForcedAligner files (src/forced_aligner.cpp:136-175): converter keys
        # only, aligner defaults; classify head output.weight
        self.aligner = "qwen3-asr.classify_num" in kv or "output.weight" in g.tensors
        if self.aligner:
            m.aligner = 1
            m.enc_layers = int(kv.get("qwen3-asr.audio.encoder.layer_count", 24))
            m.d_model = int(kv.get("qwen3-asr.audio.encoder.embedding_length", 1024))
            m.enc_heads = int(kv.get("qwen3-asr.audio.encoder.attention.head_count", 16))
            m.enc_ffn = int(kv.get("qwen3-asr.audio.encoder.feed_forward_length", 4096))
            m.conv_ch = int(kv.get("qwen3-asr.audio.conv_channels", 480))
        else:
            m.enc_layers = k2("audio.encoder_layers", "qwen3-asr.audio.encoder.layer_count", 18)
            m.d_model = k2("audio.d_model", "qwen3-asr.audio.encoder.embedding_length", 896)
            m.enc_heads = k2("audio.attention_heads", "qwen3-asr.audio.encoder.attention.head_count", 14)
            m.enc_ffn = k2("audio.ffn_dim", "qwen3-asr.audio.encoder.feed_forward_length", 3584)
            m.conv_ch = k2("audio.conv_channels", "qwen3-asr.audio.conv_channels", 480)
        m.n_mel = 128
        m.enc_eps = 1e-5
        m.vocab = int(kv.get("qwen3-asr.vocab_size", 152064 if self.aligner else 151936))
        m.hidden = int(kv.get("qwen3-asr.embedding_length", 1024))
        m.dec_layers = int(kv.get("qwen3-asr.block_count", 28))
        m.n_head = int(kv.get("qwen3-asr.attention.head_count", 16))
        m.n_kv_head = int(kv.get("qwen3-asr.attention.head_count_kv", 8))
        m.head_dim = int(kv.get("qwen3-asr.attention.key_length", 128))
        m.dec_ffn = int(kv.get("qwen3-asr.feed_forward_length", 3072))
        m.rms_eps = float(kv.get("qwen3-asr.attention.layer_norm_rms_epsilon", 1e-6))
        m.rope_theta = float(kv.get("qwen3-asr.rope.freq_base", 1e6))
        m.eos_id = 151645
        m.audio_start_id = int(kv.get("qwen3-asr.audio.start_token_id", 151669))
        m.audio_end_id = int(kv.get("qwen3-asr.audio.end_token_id", 151670))
        m.audio_pad_id = int(kv.get("qwen3-asr.audio.pad_token_id", 151676))
        self._keep = []
        # linear 2-D weights share one type: F16 (1) or Q8_0 (8); convs and
        # token_embd stay F16 (scripts/convert_hf_to_gguf.py:230-308)
        m.wtype = g.tensors["blk.0.attn_q.weight"][0]
        self.wtype = m.wtype

        def ptr(name, linear=False):
            ty, ne, arr = g.tensors[name]
            if linear and ty != m.wtype:
                raise ValueError(f"{name}: mixed linear weight types")
            if not linear and ty == 8:
                raise ValueError(f"{name}: Q8_0 only for linear weights")
            a = np.ascontiguousarray(arr)
            self._keep.append(a)
            return a.ctypes.data

        e = "audio.encoder."
        m.conv1_w, m.conv2_w, m.conv3_w = ptr(e + "conv1.weight"), ptr(e + "conv2.weight"), ptr(e + "conv3.weight")
        m.conv1_b, m.conv2_b, m.conv3_b = ptr(e + "conv1.bias"), ptr(e + "conv2.bias"), ptr(e + "conv3.bias")
        m.conv_out_w = ptr(e + "conv_out.weight", True)
        m.ln_post_w, m.ln_post_b = ptr(e + "ln_post.weight"), ptr(e + "ln_post.bias")
        m.proj1_w, m.proj1_b = ptr(e + "proj1.weight", True), ptr(e + "proj1.bias")
        m.proj2_w, m.proj2_b = ptr(e + "proj2.weight", True), ptr(e + "proj2.bias")
        self.enc = (EncLayer * m.enc_layers)()
        for i in range(m.enc_layers):
            p = f"{e}blk.{i}."
            L = self.enc[i]
            for f, n in (("attn_q_w", "attn_q.weight"), ("attn_k_w", "attn_k.weight"), ("attn_v_w", "attn_v.weight"),
                         ("attn_out_w", "attn_out.weight"), ("attn_q_b", "attn_q.bias"), ("attn_k_b", "attn_k.bias"),
                         ("attn_v_b", "attn_v.bias"), ("attn_out_b", "attn_out.bias"), ("attn_norm_w", "attn_norm.weight"),
                         ("attn_norm_b", "attn_norm.bias"), ("ffn_up_w", "ffn_up.weight"), ("ffn_down_w", "ffn_down.weight"),
                         ("ffn_up_b", "ffn_up.bias"), ("ffn_down_b", "ffn_down.bias"), ("ffn_norm_w", "ffn_norm.weight"),
                         ("ffn_norm_b", "ffn_norm.bias")):
                setattr(L, f, ptr(p + n, f in ("attn_q_w", "attn_k_w", "attn_v_w", "attn_out_w", "ffn_up_w", "ffn_down_w")))
        m.enc = self.enc
        m.token_embd = ptr("token_embd.weight")
        m.output_norm = ptr("output_norm.weight")
        self.dec = (DecLayer * m.dec_layers)()
        for i in range(m.dec_layers):
            p = f"blk.{i}."
            L = self.dec[i]
            for f in ("attn_norm", "attn_q_norm", "attn_k_norm", "ffn_norm", "attn_q", "attn_k", "attn_v", "attn_output",
                      "ffn_gate", "ffn_up", "ffn_down"):
                setattr(L, f, ptr(p + f + ".weight", f in ("attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up",
                                                           "ffn_down")))
        m.dec = self.dec
        if self.aligner:
            m.classify_num = int(kv.get("qwen3-asr.classify_num", 5000))
            self.timestamp_id = int(kv.get("qwen3-asr.timestamp_token_id", 151705))
            ty, ne, arr = g.tensors["output.weight"]
            assert ty == 1 and ne[0] == m.hidden and ne[1] >= m.classify_num
            a = np.ascontiguousarray(arr[:m.classify_num * m.hidden])   # first classify_num rows (:274-277)
            self._keep.append(a)
            m.classify_w = a.ctypes.data
        self.m = m
        self.vocab = m.vocab
        self.hidden = m.hidden

    @staticmethod
    def frames(T: int, flags: int = 0) -> int:
        if flags & OracleModel.ENC_NO_CHUNK:   # src/audio_encoder.cpp:304-310 over the whole length
            for _ in range(3):
                T = (T - 1) // 2 + 1
            return T
        return olib().qo_enc_frames(T)

    def encode(self, mel: np.ndarray, flags: int = 0) -> np.ndarray:
        mel = np.ascontiguousarray(mel, np.float32)
        T = mel.shape[1]
        N = self.frames(T, flags)
        out = np.zeros(max(1, N * self.hidden), np.float32)
        olib().qo_encode(C.byref(self.m), _f(mel), T, _f(out), flags)
        return out[:N * self.hidden].reshape(N, self.hidden)

    def encode_conv(self, mel: np.ndarray, flags: int = 0) -> np.ndarray:
        mel = np.ascontiguousarray(mel, np.float32)
        T = mel.shape[1]
        N = self.frames(T, flags)
        D = self.m.d_model
        out = np.zeros(max(1, N * D), np.float32)
        olib().qo_encode_conv(C.byref(self.m), _f(mel), T, _f(out), flags)
        return out[:N * D].reshape(N, D)

    def prompt(self, n_audio: int) -> np.ndarray:
        P = olib().qo_build_prompt(C.byref(self.m), n_audio, None)
        ids = np.zeros(P, np.int32)
        olib().qo_build_prompt(C.byref(self.m), n_audio, ids.ctypes.data_as(C.POINTER(C.c_int32)))
        return ids

    def transcribe(self, pcm, max_tokens=64, ignore_eos=False, flags=0):
        pcm = np.ascontiguousarray(pcm, np.float32)
        toks = np.zeros(max_tokens, np.int32)
        t = np.zeros(3, np.float64)
        n = olib().qo_transcribe(C.byref(self.m), _f(pcm), len(pcm), max_tokens, int(ignore_eos), flags,
                                 toks.ctypes.data_as(C.POINTER(C.c_int32)), t.ctypes.data_as(C.POINTER(C.c_double)))
        return toks[:max(n, 0)].tolist(), t


    # ------------------------------------------------------------ aligner
    def align_forward(self, tokens, audio, audio_pos, rows, flags=0):
        """ForcedAligner::forward_decoder + classify head at `rows` -> logits[len(rows)][classify_num]."""
        toks = np.ascontiguousarray(tokens, np.int32)
        a = np.ascontiguousarray(audio, np.float32)
        r = np.ascontiguousarray(rows, np.int32)
        out = np.zeros((max(len(r), 1), self.m.classify_num), np.float32)
        rc = olib().qo_align_forward(C.byref(self.m), toks.ctypes.data_as(C.POINTER(C.c_int32)), len(toks), _f(a),
                                     a.shape[0], audio_pos, r.ctypes.data_as(C.POINTER(C.c_int)), len(r), _f(out), flags)
        assert rc == 0
        return out[:len(r)]

    def align_classes(self, pcm, text_ids, flags=0):
        """ForcedAligner::align up to extract_timestamp_classes (src/forced_aligner.cpp:1636-1690):
        returns (classes, logits at the timestamp rows, tokens)."""
        mel = log_mel(pcm)
        feats = self.encode(mel, flags)
        T = mel.shape[1]
        leave = T % 100
        feat = (leave - 1) // 2 + 1 if leave > 0 else 1      # C integer division of (0-1)/2 = 0
        pads = ((feat - 1) // 2 + 1 - 1) // 2 + 1 + (T // 100) * 13
        toks = [self.m.audio_start_id] + [self.m.audio_pad_id] * pads + [self.m.audio_end_id] + list(text_ids)
        rows = [i for i, t in enumerate(toks) if t == self.timestamp_id]
        lg = self.align_forward(toks, feats, 1, rows, flags)
        cls = [int(olib().qo_argmax(_f(np.ascontiguousarray(l)), len(l))) for l in lg]
        return cls, lg, toks


class OracleDecoder:
    def __init__(self, om: OracleModel, n_ctx: int, flags: int = 0):
        self.om = om
        self.h = olib().qo_dec_new(C.byref(om.m), n_ctx, flags)

    def __del__(self):
        try:
            olib().qo_dec_free(self.h)
        except Exception:
            pass

    def forward(self, tokens, n_past, audio=None, audio_pos=-1):
        toks = np.ascontiguousarray(tokens, np.int32)
        logits = np.zeros(self.om.vocab, np.float32)
        a = None if audio is None else np.ascontiguousarray(audio, np.float32)
        rc = olib().qo_dec_forward(self.h, toks.ctypes.data_as(C.POINTER(C.c_int32)), len(toks),
                                   _f(a) if a is not None else None, 0 if a is None else a.shape[0], audio_pos, n_past,
                                   _f(logits))
        assert rc == 0
        return logits


# --------------------------------------------------------- reference (built)
_rlib = None


def have_ref() -> bool:
    return os.path.exists(REF_LIB)


def rlib():
    global _rlib
    if _rlib is None:
        L = C.CDLL(REF_LIB)
        F, I = C.POINTER(C.c_float), C.c_int
        L.ref_mel_filters.argtypes = [F]
        L.ref_log_mel.argtypes = [F, I, F]
        L.ref_log_mel.restype = I
        L.ref_load_wav.argtypes = [C.c_char_p, F, I, C.POINTER(I)]
        L.ref_inject_audio.argtypes = [C.POINTER(C.c_int32), I, F, I, F, I, I, C.c_int32, F]
        _rlib = L
    return _rlib


def ref_log_mel(pcm: np.ndarray) -> np.ndarray:
    pcm = np.ascontiguousarray(pcm, np.float32)
    T = rlib().ref_log_mel(_f(pcm), len(pcm), None)
    out = np.zeros(max(1, 128 * T), np.float32)
    rlib().ref_log_mel(_f(pcm), len(pcm), _f(out))
    return out[:128 * T].reshape(128, T)


def ref_mel_filters() -> np.ndarray:
    out = np.zeros(128 * 201, np.float32)
    rlib().ref_mel_filters(_f(out))
    return out.reshape(128, 201)
