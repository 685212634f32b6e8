"""qasr -- ctypes binding of libqasr.so (include/qasr_capi.h).

Host-side mirror of the reference's Qwen3ASR / AudioEncoder / TextDecoder
surface (src/qwen3_asr.h:55-116, src/audio_encoder.h:27-33,
src/text_decoder.h:116-137) for tests, bench and scripting.  Every call goes
through the C-ABI into hand-written HIP kernels; there is no CPU fallback:
loading fails loudly if the in-tree libqasr.so is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("QASR_LIB_OVERRIDE") or os.path.join(PKG_DIR, "libqasr.so")   # (override: diagnostic builds only)

EXPORTS = [
    "qasr_last_error", "qasr_version", "qasr_device_count", "qasr_check_expf_nonpos",
    "qasr_model_load", "qasr_model_free", "qasr_model_hparams", "qasr_model_device_bytes",
    "qasr_ctx_create", "qasr_ctx_free",
    "qasr_mel_frames", "qasr_encoder_frames", "qasr_prompt_len", "qasr_build_prompt",
    "qasr_mel", "qasr_encode", "qasr_encode_conv", "qasr_encode_no_chunk", "qasr_encoder_frames_no_chunk",
    "qasr_prefill", "qasr_prefill_chunk", "qasr_prefill_chunk_audio", "qasr_decode_step",
    "qasr_stage_audio", "qasr_run", "qasr_run_staged", "qasr_run_stream", "qasr_run_stream_staged", "qasr_set_system_prompt", "qasr_transcribe_batch",
    "qasr_set_probe", "qasr_get_probe", "qasr_get_probe_device",
    "qasr_ctx_set_option", "qasr_ctx_get_option", "qasr_debug_read",
    "qasr_set_token_callback", "qasr_set_profile", "qasr_profile_report",
    "qasr_detokenize", "qasr_tokenize",
    "qasr_load_wav", "qasr_write_wav", "qasr_synth_pcm", "qasr_write_synthetic_gguf", "qasr_synthetic_gguf_version",
    "qasr_align", "qasr_align_tokenize", "qasr_model_load_korean_dict", "qasr_fix_timestamps",
    "qasr_align_prompt_len", "qasr_align_json", "qasr_align_json_batch", "qasr_align_words",
    "qasr_ctx_grow_shape",
]


class Hparams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("enc_layers", "d_model", "enc_heads", "enc_ffn", "conv_channels", "n_mel")] + [
        ("enc_eps", C.c_float)] + [(n, C.c_int32) for n in (
            "vocab_size", "hidden_size", "dec_layers", "n_heads", "n_kv_heads", "head_dim", "dec_ffn")] + [
        ("rms_eps", C.c_float), ("rope_theta", C.c_float)] + [(n, C.c_int32) for n in (
            "eos_id", "pad_id", "audio_start_id", "audio_end_id", "audio_pad_id", "weight_type",
            "classify_num", "timestamp_token_id")]


class Timings(C.Structure):
    _fields_ = [("t_mel_ms", C.c_double), ("t_encode_ms", C.c_double), ("t_prefill_ms", C.c_double),
                ("t_decode_ms", C.c_double), ("t_total_ms", C.c_double), ("n_decode_steps", C.c_int32)]


class StreamStats(C.Structure):
    _fields_ = [("n_clips", C.c_int32), ("n_errors", C.c_int32), ("n_prefills", C.c_int32), ("n_steps", C.c_int64),
                ("slot_steps", C.c_int64), ("live_steps", C.c_int64), ("t_prefill_ms", C.c_double),
                ("t_decode_ms", C.c_double), ("t_total_ms", C.c_double), ("t_mel_ms", C.c_double),
                ("t_encode_ms", C.c_double), ("kv_keys", C.c_int64)]


_lib = None
# void (*)(void *user, int seq, int n_generated, int32_t token)
TOKEN_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int32)
# int (*)(void *user, const float **pcm, int *n_samples, int *max_tokens)
FETCH_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int), C.POINTER(C.c_int))
# int (*)(void *user, int *max_tokens)
FETCH_STAGED_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int))
# void (*)(void *user, int id, int status, const int32_t *tokens, int n_tokens)
SINK_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int32), C.c_int)


def lib() -> C.CDLL:
    """Load the in-tree libqasr.so (raises if it was not built).  A process
    that also uses torch's HIP (torch.distributed over RCCL) initialises that
    first: torch bundles its own libamdhip64 / libhsa-runtime, which
    libqasr.so then binds to by soname; loaded before them, two HSA runtimes
    end up in one process and torch's, initialised second, sees no device
    (or the other way round)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libqasr.so not built at {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        P, I, F = C.c_void_p, C.c_int, C.POINTER(C.c_float)
        I32P, IP = C.POINTER(C.c_int32), C.POINTER(C.c_int)
        sig = {
            "qasr_last_error": ([], C.c_char_p), "qasr_version": ([], C.c_char_p),
            "qasr_device_count": ([IP], I),
            "qasr_check_expf_nonpos": ([I, C.POINTER(C.c_uint64)], I),
            "qasr_model_load": ([C.c_char_p, I, C.POINTER(P)], I), "qasr_model_free": ([P], None),
            "qasr_model_hparams": ([P, C.POINTER(Hparams)], I), "qasr_model_device_bytes": ([P], C.c_int64),
            "qasr_ctx_create": ([P, I, I, C.POINTER(P)], I), "qasr_ctx_free": ([P], None),
            "qasr_mel_frames": ([I], I), "qasr_encoder_frames": ([I], I), "qasr_prompt_len": ([I], I),
            "qasr_build_prompt": ([P, I, I32P, IP], I),
            "qasr_mel": ([P, C.POINTER(F), IP, I, F], I),
            "qasr_encode": ([P, F, IP, I, F], I), "qasr_encode_conv": ([P, F, IP, I, F], I),
            "qasr_encode_no_chunk": ([P, F, IP, I, F], I), "qasr_encoder_frames_no_chunk": ([I], I),
            "qasr_prefill": ([P, I32P, IP, F, IP, IP, I, F, I32P], I),
            "qasr_decode_step": ([P, I32P, IP, I, F, I32P], I),
            "qasr_prefill_chunk": ([P, I32P, IP, IP, I, F, I32P], I),
            "qasr_prefill_chunk_audio": ([P, I32P, IP, IP, F, IP, IP, I, F, I32P], I),
            "qasr_stage_audio": ([P, C.POINTER(F), IP, I], I),
            "qasr_run": ([P, I, I, I32P, IP, C.POINTER(Timings)], I),
            "qasr_run_staged": ([P, IP, I, I, I, I32P, IP, C.POINTER(Timings)], I),
            "qasr_run_stream": ([P, I, FETCH_FN, SINK_FN, P, I, I, C.POINTER(StreamStats)], I),
            "qasr_run_stream_staged": ([P, I, FETCH_STAGED_FN, SINK_FN, P, I, I, C.POINTER(StreamStats)], I),
            "qasr_set_system_prompt": ([P, I32P, I], I),
            "qasr_transcribe_batch": ([P, C.POINTER(F), IP, I, I, I, I32P, IP, C.POINTER(Timings)], I),
            "qasr_set_probe": ([P, I], I),
            "qasr_get_probe": ([P, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_double)], I),
            "qasr_get_probe_device": ([P, C.POINTER(C.c_double), C.POINTER(C.c_int64)], I),
            "qasr_ctx_set_option": ([P, C.c_char_p, I], I), "qasr_ctx_get_option": ([P, C.c_char_p, IP], I),
            "qasr_debug_read": ([P, C.c_char_p, P, C.c_int64], I),
            "qasr_set_token_callback": ([P, TOKEN_CB, P], I),
            "qasr_set_profile": ([P, I], I), "qasr_profile_report": ([P, C.c_char_p, I], I),
            "qasr_detokenize": ([P, I32P, I, C.c_char_p, I], I), "qasr_tokenize": ([P, C.c_char_p, I32P, I], I),
            "qasr_load_wav": ([C.c_char_p, F, I, IP], I), "qasr_write_wav": ([C.c_char_p, F, I, I], I),
            "qasr_synth_pcm": ([C.c_uint64, I, F], I),
            "qasr_write_synthetic_gguf": ([C.c_char_p, C.c_char_p, C.c_uint64, I], I),
            "qasr_synthetic_gguf_version": ([], I),
            "qasr_align": ([P, F, I, I32P, I, I32P, I, IP, C.POINTER(Timings)], I),
            "qasr_align_tokenize": ([P, C.c_char_p, C.c_char_p, I32P, I, IP], I),
            "qasr_model_load_korean_dict": ([P, C.c_char_p], I),
            "qasr_fix_timestamps": ([I32P, I, I32P], I),
            "qasr_ctx_grow_shape": ([I, I, I, I, IP, IP], None),
            "qasr_align_prompt_len": ([I, I], I),
            "qasr_align_words": ([P, C.c_char_p, C.c_char_p, C.c_char_p, I], I),
            "qasr_align_json": ([P, F, I, C.c_char_p, C.c_char_p, C.c_char_p, I, C.POINTER(Timings)], I),
            "qasr_align_json_batch": ([P, C.POINTER(F), IP, C.POINTER(C.c_char_p), I, C.c_char_p, C.c_char_p, I,
                                       C.POINTER(Timings)], I),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


class QasrError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise QasrError(f"{what}: {lib().qasr_last_error().decode(errors='replace')}")


def _f(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i32(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _i(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int))


# ------------------------------------------------------------------ host utils
def mel_frames(n: int) -> int:
    return lib().qasr_mel_frames(n)


def encoder_frames(T: int) -> int:
    return lib().qasr_encoder_frames(T)


def synth_pcm(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    _check(lib().qasr_synth_pcm(seed, n, _f(out)), "synth_pcm")
    return out


def write_synthetic_gguf(path: str, config: str = "tiny", seed: int = 42, wtype: int = 1) -> None:
    _check(lib().qasr_write_synthetic_gguf(path.encode(), config.encode(), seed, wtype), "write_synthetic_gguf")


def load_wav(path: str):
    sr = C.c_int(0)
    n = lib().qasr_load_wav(path.encode(), None, 0, C.byref(sr))
    if n < 0:
        raise QasrError(f"load_wav: {lib().qasr_last_error().decode()}")
    out = np.zeros(n, np.float32)
    lib().qasr_load_wav(path.encode(), _f(out), n, C.byref(sr))
    return out, sr.value


def write_wav(path: str, pcm: np.ndarray, sr: int = 16000) -> None:
    pcm = np.ascontiguousarray(pcm, np.float32)
    _check(lib().qasr_write_wav(path.encode(), _f(pcm), len(pcm), sr), "write_wav")


def fix_timestamps(classes: Sequence[int]) -> List[int]:
    """LIS repair of raw timestamp classes (src/forced_aligner.cpp:1183-1265)."""
    a = np.ascontiguousarray(classes, np.int32)
    out = np.zeros(max(len(a), 1), np.int32)
    _check(lib().qasr_fix_timestamps(_i32(a) if len(a) else None, len(a), _i32(out) if len(a) else None), "fix_timestamps")
    return out[:len(a)].tolist()


def align_prompt_len(n_samples: int, n_text: int) -> int:
    return lib().qasr_align_prompt_len(n_samples, n_text)


def device_count() -> int:
    n = C.c_int(0)
    lib().qasr_device_count(C.byref(n))
    return n.value


# ---------------------------------------------------------------------- model
class Model:
    """qasr_model: weights in one device arena (src/qwen3_asr.cpp:21-42)."""

    def __init__(self, path: str, device: int = 0):
        self.h = C.c_void_p()
        _check(lib().qasr_model_load(path.encode(), device, C.byref(self.h)), "qasr_model_load")
        hp = Hparams()
        _check(lib().qasr_model_hparams(self.h, C.byref(hp)), "qasr_model_hparams")
        self.hp = hp
        self.path = path

    def close(self):
        if self.h:
            lib().qasr_model_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_bytes(self) -> int:
        return lib().qasr_model_device_bytes(self.h)

    def build_prompt(self, n_audio: int):
        P = lib().qasr_prompt_len(n_audio)
        ids = np.zeros(P, np.int32)
        pos = C.c_int(0)
        lib().qasr_build_prompt(self.h, n_audio, _i32(ids), C.byref(pos))
        return ids, pos.value

    def detokenize(self, ids: Sequence[int]) -> str:
        a = np.ascontiguousarray(ids, np.int32)
        n = lib().qasr_detokenize(self.h, _i32(a), len(a), None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().qasr_detokenize(self.h, _i32(a), len(a), buf, n + 1)
        return buf.raw[:n].decode("utf-8", errors="replace")

    def tokenize(self, text: str) -> List[int]:
        n = lib().qasr_tokenize(self.h, text.encode(), None, 0)
        a = np.zeros(max(n, 1), np.int32)
        lib().qasr_tokenize(self.h, text.encode(), _i32(a), n)
        return a[:n].tolist()


    # ---- forced aligner (Qwen3-ForcedAligner files) -------------------------
    @property
    def is_aligner(self) -> bool:
        return self.hp.classify_num > 0

    def align_tokenize(self, text: str, language: str = ""):
        """ForcedAligner::tokenize_with_timestamps -> (ids, n_words)."""
        nw = C.c_int(0)
        n = lib().qasr_align_tokenize(self.h, text.encode(), language.encode(), None, 0, C.byref(nw))
        a = np.zeros(max(n, 1), np.int32)
        lib().qasr_align_tokenize(self.h, text.encode(), language.encode(), _i32(a), n, C.byref(nw))
        return a[:n].tolist(), nw.value

    def align_words(self, text: str, language: str = "") -> List[str]:
        n = lib().qasr_align_words(self.h, text.encode(), language.encode(), None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().qasr_align_words(self.h, text.encode(), language.encode(), buf, n + 1)
        s = buf.raw[:n].decode("utf-8")
        return s.split("\n") if s else []

    def load_korean_dict(self, path: str) -> None:
        _check(lib().qasr_model_load_korean_dict(self.h, path.encode()), "qasr_model_load_korean_dict")


@dataclass
class RunResult:
    tokens: List[List[int]]
    timings: Timings


def _sink_into(out: dict, failed: list):
    def sink(_u, cid, status, toks, n):
        try:
            if status:
                out[cid] = QasrError(lib().qasr_last_error().decode(errors="replace"))
            else:
                out[cid] = [int(toks[i]) for i in range(n)]
        except BaseException as e:   # (ctypes would swallow it)
            failed.append(e)
    return sink


def _guarded_fetch(fetch, failed: list):
    """A ctypes callback cannot raise: an exception in next_clip() (e.g. a
    TCPStore failure of the shared queue) is stored, the queue reported empty
    (-1, so the engine drains its slots and returns), and the caller re-raises
    it after the run instead of the engine taking 0 as a clip id."""
    def f(*a):
        if failed:
            return -1
        try:
            return fetch(*a)
        except BaseException as e:
            failed.append(e)
            return -1
    return f


class Context:
    """qasr_ctx: stream, KV cache, scratch (TextDecoder::init_kv_cache analogue)."""

    def __init__(self, model: Model, max_batch: int = 1, max_ctx: int = 2048):
        self.model = model
        self.h = C.c_void_p()
        _check(lib().qasr_ctx_create(model.h, max_batch, max_ctx, C.byref(self.h)), "qasr_ctx_create")
        self.max_batch, self.max_ctx = max_batch, max_ctx

    def close(self):
        if self.h:
            lib().qasr_ctx_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- stages ------------------------------------------------------------
    def mel(self, clips: Sequence[np.ndarray]) -> List[np.ndarray]:
        clips = [np.ascontiguousarray(c, np.float32) for c in clips]
        n = np.array([len(c) for c in clips], np.int32)
        T = [mel_frames(int(k)) for k in n]
        out = np.zeros(max(1, 128 * sum(T)), np.float32)
        ptrs = (C.POINTER(C.c_float) * len(clips))(*[_f(c) for c in clips])
        _check(lib().qasr_mel(self.h, ptrs, _i(n), len(clips), _f(out)), "qasr_mel")
        res, o = [], 0
        for t in T:
            res.append(out[o:o + 128 * t].reshape(128, t))
            o += 128 * t
        return res

    def _encode(self, mels: Sequence[np.ndarray], conv_only: bool, no_chunk: bool = False) -> List[np.ndarray]:
        T = np.array([m.shape[1] for m in mels], np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.ascontiguousarray(m, np.float32).ravel() for m in mels]))
        N = [lib().qasr_encoder_frames_no_chunk(int(t)) if no_chunk else encoder_frames(int(t)) for t in T]
        width = self.model.hp.d_model if conv_only else self.model.hp.hidden_size
        out = np.zeros(max(1, sum(N) * width), np.float32)
        fn = lib().qasr_encode_no_chunk if no_chunk else lib().qasr_encode_conv if conv_only else lib().qasr_encode
        _check(fn(self.h, _f(flat), _i(T), len(mels), _f(out)), "qasr_encode")
        res, o = [], 0
        for k in N:
            res.append(out[o * width:(o + k) * width].reshape(k, width))
            o += k
        return res

    def encode(self, mels):
        return self._encode(mels, False)

    def encode_no_chunk(self, mels):
        """AudioEncoder::encode_no_chunk: the conv stack over all frames at once, PE 0..N-1"""
        return self._encode(mels, False, True)

    def encode_conv(self, mels):
        return self._encode(mels, True)

    def prefill(self, ids_list, feats_list=None, audio_pos=None, want_logits=True):
        B = len(ids_list)
        P = np.array([len(x) for x in ids_list], np.int32)
        ids = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int32) for x in ids_list]))
        feats = None
        N = np.zeros(B, np.int32)
        ap = np.full(B, -1, np.int32) if audio_pos is None else np.asarray(audio_pos, np.int32)
        if feats_list is not None:
            N = np.array([f.shape[0] for f in feats_list], np.int32)
            feats = np.ascontiguousarray(np.concatenate([np.asarray(f, np.float32) for f in feats_list]))
        V = self.model.hp.vocab_size
        logits = np.zeros((B, V), np.float32) if want_logits else None
        am = np.zeros(B, np.int32)
        _check(lib().qasr_prefill(self.h, _i32(ids), _i(P), _f(feats) if feats is not None else None, _i(ap), _i(N), B,
                                  _f(logits) if want_logits else None, _i32(am)), "qasr_prefill")
        return logits, am

    def decode_step(self, tok, n_past, want_logits=True):
        tok = np.ascontiguousarray(tok, np.int32)
        npast = np.ascontiguousarray(n_past, np.int32)
        B = len(tok)
        logits = np.zeros((B, self.model.hp.vocab_size), np.float32) if want_logits else None
        am = np.zeros(B, np.int32)
        _check(lib().qasr_decode_step(self.h, _i32(tok), _i(npast), B, _f(logits) if want_logits else None, _i32(am)),
               "qasr_decode_step")
        return logits, am

    def prefill_chunk(self, ids_list, n_past, want_logits=True, feats_list=None, audio_pos=None):
        """qasr_prefill_chunk: sequence b's tokens ids_list[b] after n_past[b]
        cached ones, one causal chunk (TextDecoder::forward, n_tokens > 1);
        with feats_list / audio_pos: qasr_prefill_chunk_audio, the audio rows
        spliced at audio_pos[b] of the chunk (forward_with_audio at n_past > 0);
        returns (logits of each chunk's last row, argmax)"""
        P = np.array([len(x) for x in ids_list], np.int32)
        ids = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int32) for x in ids_list]), np.int32)
        npast = np.ascontiguousarray(n_past, np.int32)
        B = len(P)
        logits = np.zeros((B, self.model.hp.vocab_size), np.float32) if want_logits else None
        am = np.zeros(B, np.int32)
        if feats_list is None:
            _check(lib().qasr_prefill_chunk(self.h, _i32(ids), _i(P), _i(npast), B, _f(logits) if want_logits else None,
                                            _i32(am)), "qasr_prefill_chunk")
            return logits, am
        N = np.array([f.shape[0] for f in feats_list], np.int32)
        feats = np.ascontiguousarray(np.concatenate([np.asarray(f, np.float32) for f in feats_list]))
        ap = np.ascontiguousarray(audio_pos, np.int32)
        _check(lib().qasr_prefill_chunk_audio(self.h, _i32(ids), _i(P), _i(npast), _f(feats), _i(ap), _i(N), B,
                                              _f(logits) if want_logits else None, _i32(am)), "qasr_prefill_chunk_audio")
        return logits, am

    # ---- whole path --------------------------------------------------------
    def stage_audio(self, clips: Sequence[np.ndarray]) -> None:
        self._staged = [np.ascontiguousarray(c, np.float32) for c in clips]
        n = np.array([len(c) for c in self._staged], np.int32)
        ptrs = (C.POINTER(C.c_float) * len(self._staged))(*[_f(c) for c in self._staged])
        _check(lib().qasr_stage_audio(self.h, ptrs, _i(n), len(self._staged)), "qasr_stage_audio")

    def run(self, max_tokens: int, ignore_eos: bool = False) -> RunResult:
        B = len(self._staged)
        if B > self.max_batch:
            raise QasrError(f"{B} staged clips exceed max_batch {self.max_batch}: use run_staged")
        toks = np.zeros((B, max_tokens), np.int32)
        nt = np.zeros(B, np.int32)
        t = Timings()
        _check(lib().qasr_run(self.h, max_tokens, int(ignore_eos), _i32(toks), _i(nt), C.byref(t)), "qasr_run")
        return RunResult([toks[b, :nt[b]].tolist() for b in range(B)], t)

    def run_staged(self, clips: Sequence[int], max_tokens: int, ignore_eos: bool = False) -> RunResult:
        """transcribe staged clips (indices into the last stage_audio call) as one batch"""
        idx = np.ascontiguousarray(clips, np.int32)
        B = len(idx)
        toks = np.zeros((B, max_tokens), np.int32)
        nt = np.zeros(B, np.int32)
        t = Timings()
        _check(lib().qasr_run_staged(self.h, _i(idx), B, max_tokens, int(ignore_eos), _i32(toks), _i(nt), C.byref(t)),
               "qasr_run_staged")
        return RunResult([toks[b, :nt[b]].tolist() for b in range(B)], t)

    def run_stream(self, next_clip, max_tokens: int, ignore_eos: bool = False, slots: int = 0):
        """Continuous batching (qasr_run_stream): next_clip() -> (id, pcm[, budget])
        or None when the queue is empty; returns ({id: tokens | QasrError},
        StreamStats).  Slots (0: max_batch) freed by a finished clip are
        refilled at the next chunk boundary; a clip that fails alone maps to
        its QasrError."""
        out, keep = {}, []

        def fetch(_u, pcm_pp, n_p, budget_p):
            item = next_clip()
            if item is None:
                return -1
            cid, pcm = int(item[0]), np.ascontiguousarray(item[1], np.float32)
            keep[:] = [pcm]   # alive until the next fetch (the engine copies it first)
            pcm_pp[0] = _f(pcm)
            n_p[0] = len(pcm)
            if len(item) > 2:
                budget_p[0] = int(item[2])
            return cid

        failed = []
        f, k = FETCH_FN(_guarded_fetch(fetch, failed)), SINK_FN(_sink_into(out, failed))
        st = StreamStats()
        rc = lib().qasr_run_stream(self.h, int(slots), f, k, None, int(max_tokens), int(ignore_eos), C.byref(st))
        if failed:
            raise failed[0]
        _check(rc, "qasr_run_stream")
        return out, st

    def run_stream_staged(self, next_clip, max_tokens: int, ignore_eos: bool = False, slots: int = 0):
        """run_stream over the staged pool (stage_audio): next_clip() -> staged
        index (its id) or (index, budget), None when the queue is empty"""
        out = {}

        def fetch(_u, budget_p):
            item = next_clip()
            if item is None:
                return -1
            if isinstance(item, tuple):
                budget_p[0] = int(item[1])
                return int(item[0])
            return int(item)

        failed = []
        f, k = FETCH_STAGED_FN(_guarded_fetch(fetch, failed)), SINK_FN(_sink_into(out, failed))
        st = StreamStats()
        rc = lib().qasr_run_stream_staged(self.h, int(slots), f, k, None, int(max_tokens), int(ignore_eos), C.byref(st))
        if failed:
            raise failed[0]
        _check(rc, "qasr_run_stream_staged")
        return out, st

    def set_system_prompt(self, ids: Sequence[int]) -> None:
        a = np.ascontiguousarray(ids, np.int32)
        _check(lib().qasr_set_system_prompt(self.h, _i32(a) if len(a) else None, len(a)), "qasr_set_system_prompt")

    def set_option(self, name: str, value: int) -> None:
        _check(lib().qasr_ctx_set_option(self.h, name.encode(), int(value)), "qasr_ctx_set_option")

    def get_option(self, name: str) -> int:
        v = C.c_int(0)
        _check(lib().qasr_ctx_get_option(self.h, name.encode(), C.byref(v)), "qasr_ctx_get_option")
        return v.value

    def debug_read(self, buffer: str) -> np.ndarray:
        """Decode-step state after decode_step: x (fp32), act (fp16), qkv (fp32), att (fp16)."""
        hp = self.model.hp
        qd, kd = hp.n_heads * 128, hp.n_kv_heads * 128
        n, dt = {"x": (hp.hidden_size, np.float32), "act": (hp.dec_ffn, np.float16),
                 "qkv": (qd + 2 * kd, np.float32), "att": (qd, np.float16)}[buffer]
        out = np.zeros((self.max_batch, n), dt)
        _check(lib().qasr_debug_read(self.h, buffer.encode(), out.ctypes.data_as(C.c_void_p), out.nbytes), "qasr_debug_read")
        return out

    def set_token_callback(self, fn) -> None:
        """fn(seq, n_generated, token) after every greedy token of run() (None removes)"""
        self._tok_cb = TOKEN_CB(lambda _u, seq, n, tok: fn(seq, n, tok)) if fn else None
        _check(lib().qasr_set_token_callback(self.h, self._tok_cb if fn else TOKEN_CB(), None), "qasr_set_token_callback")

    def set_profile(self, on: bool) -> None:
        _check(lib().qasr_set_profile(self.h, int(on)), "qasr_set_profile")

    def profile_report(self) -> str:
        n = lib().qasr_profile_report(self.h, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().qasr_profile_report(self.h, buf, n + 1)
        return buf.raw[:n].decode()

    def set_probe(self, kernel: int) -> None:
        _check(lib().qasr_set_probe(self.h, kernel), "qasr_set_probe")

    def get_probe(self):
        ms, n, b = C.c_double(0), C.c_int64(0), C.c_double(0)
        _check(lib().qasr_get_probe(self.h, C.byref(ms), C.byref(n), C.byref(b)), "qasr_get_probe")
        return ms.value, n.value, b.value

    def get_probe_device(self):
        """(total ms, launches) of the probed launches by the device clock"""
        ms, n = C.c_double(0), C.c_int64(0)
        _check(lib().qasr_get_probe_device(self.h, C.byref(ms), C.byref(n)), "qasr_get_probe_device")
        return ms.value, n.value

    # ---- forced aligner ------------------------------------------------------
    def align(self, pcm: np.ndarray, text_ids: Sequence[int]):
        """Raw timestamp classes of one clip (qasr_align) -> (classes, timings)."""
        pcm = np.ascontiguousarray(pcm, np.float32)
        ids = np.ascontiguousarray(text_ids, np.int32)
        cap = max(int(np.sum(ids == self.model.hp.timestamp_token_id)), 1)
        out = np.zeros(cap, np.int32)
        nts = C.c_int(0)
        t = Timings()
        _check(lib().qasr_align(self.h, _f(pcm), len(pcm), _i32(ids) if len(ids) else None, len(ids), _i32(out), cap,
                                C.byref(nts), C.byref(t)), "qasr_align")
        return out[:nts.value].tolist(), t

    def align_json(self, pcm: np.ndarray, text: str, language: str = ""):
        """ForcedAligner::align -> the CLI JSON document (parsed) and timings.
        qasr_align_json returns the document length, or minus an error code."""
        import json
        pcm = np.ascontiguousarray(pcm, np.float32)
        t = Timings()
        cap = 8192 + 40 * len(text.encode())   # (one call in practice: the escaped words + ~50 B a word)
        buf = C.create_string_buffer(cap)
        n = lib().qasr_align_json(self.h, _f(pcm), len(pcm), text.encode(), language.encode(), buf, cap, C.byref(t))
        if n < 0:
            raise QasrError(f"qasr_align_json: {lib().qasr_last_error().decode(errors='replace')}")
        if n >= cap:   # larger than the bound: run again into a buffer of the reported size
            buf = C.create_string_buffer(n + 1)
            lib().qasr_align_json(self.h, _f(pcm), len(pcm), text.encode(), language.encode(), buf, n + 1, C.byref(t))
        return json.loads(buf.raw[:n].decode("utf-8")), t

    def align_json_batch(self, pcms, texts, language: str = ""):
        """qasr_align_json_batch: B clips in one aligner pass -> (list of the
        CLI documents, parsed, in input order; timings)"""
        import json
        arrs = [np.ascontiguousarray(p, np.float32) for p in pcms]
        B = len(arrs)
        ptrs = (C.POINTER(C.c_float) * B)(*[_f(a) for a in arrs])
        n = np.array([len(a) for a in arrs], np.int32)
        tx = (C.c_char_p * B)(*[t.encode() for t in texts])
        t = Timings()
        cap = 8192 * B + 40 * sum(len(x.encode()) for x in texts)
        buf = C.create_string_buffer(cap)
        k = lib().qasr_align_json_batch(self.h, ptrs, _i(n), tx, B, language.encode(), buf, cap, C.byref(t))
        if k < 0:
            raise QasrError(f"qasr_align_json_batch: {lib().qasr_last_error().decode(errors='replace')}")
        if k >= cap:
            buf = C.create_string_buffer(k + 1)
            lib().qasr_align_json_batch(self.h, ptrs, _i(n), tx, B, language.encode(), buf, k + 1, C.byref(t))
        return json.loads(buf.raw[:k].decode("utf-8")), t

    def transcribe(self, clips, max_tokens=1024, ignore_eos=False) -> RunResult:
        self.stage_audio(clips)
        return self.run(max_tokens, ignore_eos)
