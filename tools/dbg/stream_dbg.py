# diagnosis of qasr_run_stream refills on the tiny model (not a test)
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "qwen3-asr.cpp_amd", "python"))
import qasr, tempfile
SR = 16000
p = os.path.join(tempfile.mkdtemp(), "tiny.gguf")
qasr.write_synthetic_gguf(p, "tiny", 42, 1)
m = qasr.Model(p)
lens = [SR, 2 * SR + 333, 4 * SR, SR // 2, 3 * SR, 5 * SR + 7, SR + 999]
clips = [qasr.synth_pcm(7100 + i, n) for i, n in enumerate(lens)]

def single(pcm, b):
    c = qasr.Context(m, max_batch=1, max_ctx=640)
    r = c.transcribe([pcm], max_tokens=b, ignore_eos=True).tokens[0]
    c.close()
    return r

def batch(pcms, b, mb=3):
    c = qasr.Context(m, max_batch=mb, max_ctx=640)
    r = c.transcribe(pcms, max_tokens=b, ignore_eos=True).tokens
    c.close()
    return r

def stream(budgets, slots=3, eager=0):
    os.environ["QASR_NO_GRAPH"] = "1" if eager else "0"
    c = qasr.Context(m, max_batch=slots, max_ctx=640)
    os.environ["QASR_NO_GRAPH"] = "0"
    it = iter([(i, clips[i], b) for i, b in enumerate(budgets)])
    out, st = c.run_stream(lambda: next(it, None), max_tokens=32, ignore_eos=True)
    c.close()
    return out

ref = {i: single(clips[i], 16) for i in range(len(clips))}
print("batch(0,1,2) == single:", [batch([clips[0], clips[1], clips[2]], 16)[k] == ref[k] for k in range(3)])
print("batch(3,1,5) == single:", [a == ref[k] for a, k in zip(batch([clips[3], clips[1], clips[5]], 16), (3, 1, 5))])
for name, budgets, kw in [("fail-case", [3, 9, 5, 16, 1, 7, 12], {}), ("no-b1", [3, 9, 5, 16, 2, 7, 12], {}),
                          ("all16", [16] * 7, {}), ("fail-eager", [3, 9, 5, 16, 1, 7, 12], {"eager": 1}),
                          ("slots1", [3, 9, 5, 16, 1, 7, 12], {"slots": 1})]:
    try:
        out = stream(budgets, **kw)
    except qasr.QasrError as e:
        print(name, "error", e); continue
    bad = []
    for i, b in enumerate(budgets):
        r = ref[i][:b]
        if out[i] != r:
            k = next((j for j in range(b) if out[i][j] != r[j]), None)
            bad.append((i, k))
    print(name, "mismatch (clip, first index):", bad)
