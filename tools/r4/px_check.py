"""prefill logits of the default library against a variant (QASR_VARIANT): bit-identical?  (the exact prefill
attention's asm fast path vs the compiler's) -- full model, 92 s prompt and a 64 x 30 s batch row"""
import ctypes
import os
import subprocess
import sys
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1:   # child: one library, dump logits
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
    import bench
    import qasr
    m = qasr.Model(bench.synthetic_model(0, "full", 1))
    out = {}
    for name, secs, B in (("c1", 92, 1), ("b8", 30, 8)):
        pcm = qasr.synth_pcm(2024, secs * 16000)
        c = qasr.Context(m, max_batch=B, max_ctx=1400)
        feats = c.encode(c.mel([pcm]))[0]
        ids, pos = m.build_prompt(feats.shape[0])
        lg, _ = c.prefill([ids] * B, [feats] * B, [pos] * B)
        out[name] = np.asarray(lg)
        c.close()
    am = qasr.Model(bench.synthetic_model(0, "aligner", 1))
    ac = qasr.Context(am, max_batch=1, max_ctx=3000)
    pcm = qasr.synth_pcm(77, 40 * 16000)
    text = " ".join(["ab", "cd", "ef", "gh"] * 40)
    ids, _ = am.align_tokenize(text)
    cls, _ = ac.align(pcm, ids)
    out["align"] = np.asarray(cls)
    np.savez(sys.argv[1], **out)
    sys.exit(0)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
res = {}
for tag, lib in (("new", ""), ("old", os.environ["QASR_VARIANT"])):
    env = dict(os.environ)
    if lib:
        env["QASR_LIB_OVERRIDE"] = lib
    f = os.path.join(ROOT, "gpurun_out", f"px_{tag}.npz")
    subprocess.run([sys.executable, __file__, f], check=True, env=env, timeout=600)
    res[tag] = np.load(f)
for k in res["new"].files:
    a, b = res["new"][k], res["old"][k]
    print(k, a.shape, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a.astype(float) - b).max()}")
