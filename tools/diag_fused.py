"""Fused vs separate batch-1 decode launches, one process, per layer.

Runs one decode step of the full-size synthetic model with the decoder cut
after L layers (qasr_ctx_set_option "dec_layers") under several launch
configurations and diffs the residual stream x, the SwiGLU activation, the
raw QKV and the attention output against the separate-launch path.  Repeated
runs of one configuration show whether a difference is a race (varies run to
run) or arithmetic (fixed).

    python tools/diag_fused.py [model.gguf]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
import qasr  # noqa: E402

SEP = dict(fuse_ffn=0, fuse_qkv=0, fuse_o=0, handoff_fence=0)
CFGS = [
    ("ffn", dict(fuse_ffn=1, fuse_qkv=0, fuse_o=0, handoff_fence=0)),
    ("ffn+fence", dict(fuse_ffn=1, fuse_qkv=0, fuse_o=0, handoff_fence=1)),
    ("qkv", dict(fuse_ffn=0, fuse_qkv=1, fuse_o=0, handoff_fence=0)),
    ("qkv+fence", dict(fuse_ffn=0, fuse_qkv=1, fuse_o=0, handoff_fence=1)),
    ("qkv+o", dict(fuse_ffn=0, fuse_qkv=1, fuse_o=1, handoff_fence=0)),
    ("all", dict(fuse_ffn=1, fuse_qkv=1, fuse_o=1, handoff_fence=0)),
    ("all+fence", dict(fuse_ffn=1, fuse_qkv=1, fuse_o=1, handoff_fence=1)),
]


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/diag-full.gguf"
    if not os.path.exists(path):
        t = time.time()
        qasr.write_synthetic_gguf(path, "full", 42, 1)
        print(f"wrote {path} in {time.time() - t:.1f}s", flush=True)
    m = qasr.Model(path)
    c = qasr.Context(m, max_batch=1, max_ctx=512)
    print("slots ffn/qkv", c.get_option("slots_ffn"), c.get_option("slots_qkv"), flush=True)
    pcm = qasr.synth_pcm(14000, 3 * 16000)
    feats = c.encode(c.mel([pcm]))[0]
    ids, pos = m.build_prompt(feats.shape[0])
    c.prefill([ids], [feats], [pos])
    P = len(ids)

    def step(cfg, L):
        for k, v in cfg.items():
            c.set_option(k, v)
        c.set_option("dec_layers", L)
        lg, _ = c.decode_step([1234], [P])
        return {"x": c.debug_read("x")[0].copy(), "act": c.debug_read("act")[0].astype(np.float32),
                "qkv": c.debug_read("qkv")[0].copy(), "att": c.debug_read("att")[0].astype(np.float32),
                "logits": lg[0].copy()}

    def diff(a, b):
        d = np.abs(a - b)
        idx = np.nonzero(a != b)[0]
        return f"max {d.max():.3g} n {len(idx)}" + (f" first {idx[:6].tolist()}" if len(idx) else "")

    for L in (1, 2, 3, 28):
        base = step(SEP, L)
        again = step(SEP, L)
        same = all(np.array_equal(base[k], again[k]) for k in base)
        print(f"--- L={L}: separate repeatable: {same}", flush=True)
        for name, cfg in CFGS:
            runs = [step(cfg, L) for _ in range(6)]
            rep = all(np.array_equal(runs[0][k], r[k]) for r in runs[1:] for k in base)
            line = [f"{name:10s} repeatable={rep}"]
            for k in ("qkv", "att", "act", "x", "logits"):
                line.append(f"{k}: {diff(runs[0][k], base[k])}")
            if not rep:
                worst = max(float(np.abs(r["x"] - runs[0]["x"]).max()) for r in runs[1:])
                line.append(f"run-to-run x max {worst:.3g}")
            print("  " + " | ".join(line), flush=True)
    c.close()
    m.close()


if __name__ == "__main__":
    main()
