"""Fused vs separate batch-1 launches: staleness vs arithmetic.

(1) Token A / token B alternation at one position: a stale in-launch (or
    cross-launch) read shows up as a result that depends on the previous
    call's token.  (2) Per-layer scan: the first decoder layer whose residual
    stream differs between a fused configuration and the separate launches,
    and which elements of the SwiGLU activation / attention output differ
    there.

    python tools/diag_fused2.py [model.gguf]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
import qasr  # noqa: E402

SEP = dict(fuse_ffn=0, fuse_qkv=0, fuse_o=0)
FFN = dict(fuse_ffn=1, fuse_qkv=0, fuse_o=0)
QKV = dict(fuse_ffn=0, fuse_qkv=1, fuse_o=0)


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/diag-full.gguf"
    if not os.path.exists(path):
        qasr.write_synthetic_gguf(path, "full", 42, 1)
    m = qasr.Model(path)
    c = qasr.Context(m, max_batch=1, max_ctx=512)
    pcm = qasr.synth_pcm(14000, 3 * 16000)
    feats = c.encode(c.mel([pcm]))[0]
    ids, pos = m.build_prompt(feats.shape[0])
    c.prefill([ids], [feats], [pos])
    P = len(ids)

    def step(cfg, tok, L=0):
        for k, v in cfg.items():
            c.set_option(k, v)
        c.set_option("dec_layers", L)
        lg, _ = c.decode_step([tok], [P])
        return {"x": c.debug_read("x")[0].copy(), "act": c.debug_read("act")[0].astype(np.float32),
                "qkv": c.debug_read("qkv")[0].copy(), "att": c.debug_read("att")[0].astype(np.float32),
                "logits": lg[0].copy()}

    A, B = 1234, 98765
    seq = [("SEP", SEP, A), ("SEP", SEP, B), ("SEP", SEP, A), ("FFN", FFN, A), ("FFN", FFN, B), ("FFN", FFN, A),
           ("SEP", SEP, A), ("QKV", QKV, A), ("QKV", QKV, B), ("QKV", QKV, A), ("SEP", SEP, A), ("SEP", SEP, B)]
    res = [(n, t, step(cfg, t)) for n, cfg, t in seq]
    ref = {A: res[0][2], B: res[1][2]}
    print("--- alternation (max |logit diff| vs the first SEP result of the same token)")
    for n, t, r in res:
        d = float(np.abs(r["logits"] - ref[t]["logits"]).max())
        print(f"  {n} tok={t}: {d:.3g}", flush=True)

    print("--- per-layer scan: first layer whose x differs")
    for name, cfg in (("FFN", FFN), ("QKV", QKV)):
        for L in range(1, 29):
            s = step(SEP, A, L)
            f = step(cfg, A, L)
            if not np.array_equal(s["x"], f["x"]):
                print(f"  {name}: first differing layer index {L - 1}", flush=True)
                for k in ("qkv", "att", "act", "x"):
                    idx = np.nonzero(s[k] != f[k])[0]
                    print(f"    {k}: n {len(idx)} idx {idx[:12].tolist()}", flush=True)
                    for i in idx[:6]:
                        print(f"      [{i}] sep {s[k][i]!r} fused {f[k][i]!r}", flush=True)
                break
        else:
            print(f"  {name}: no layer differs", flush=True)
    c.close()
    m.close()


if __name__ == "__main__":
    main()
