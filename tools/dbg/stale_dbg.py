# is a clip's decode sensitive to stale KV-cache contents past its positions? (diagnosis)
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "qwen3-asr.cpp_amd", "python"))
import qasr, tempfile
import numpy as np
SR = 16000
p = os.path.join(tempfile.mkdtemp(), "tiny.gguf")
qasr.write_synthetic_gguf(p, "tiny", 42, 1)
m = qasr.Model(p)
print("hp", m.hp.hidden_size, m.hp.n_heads, m.hp.n_kv_heads, m.hp.dec_layers)
c3 = qasr.synth_pcm(7103, SR // 2)
c2 = qasr.synth_pcm(7102, 4 * SR)
for ex in (1, 0):
    c = qasr.Context(m, max_batch=1, max_ctx=640)
    c.set_option("fa_exact_decode", ex)
    a = c.transcribe([c3], max_tokens=16, ignore_eos=True).tokens[0]
    c.transcribe([c2], max_tokens=16, ignore_eos=True)
    b = c.transcribe([c3], max_tokens=16, ignore_eos=True).tokens[0]
    print("exact", ex, "fused_mode", c.get_option("fused_mode"), "fresh == dirty:", a == b, a, b)
    # teacher-forced logits: fresh vs dirty
    mel = c.mel([c3])[0]
    f = c.encode([mel])[0]
    ids, pos = m.build_prompt(f.shape[0])
    cf = qasr.Context(m, max_batch=1, max_ctx=640)
    cf.set_option("fa_exact_decode", ex)
    lf, _ = cf.prefill([ids], [f], [pos])
    ld, _ = c.prefill([ids], [f], [pos])
    print("  prefill logits equal:", np.array_equal(lf, ld))
    for k in range(10):
        t = [a[k]]
        gf, _ = cf.decode_step(t, [len(ids) + k])
        gd, _ = c.decode_step(t, [len(ids) + k])
        if not np.array_equal(gf, gd):
            print("  step", k, "differs: max", float(np.abs(gf - gd).max()))
            break
    else:
        print("  10 decode steps bit-identical")
    cf.close()
    c.close()
