"""Oracle sensitivity to the single-rounding fp16 V accumulator (QO_FA_V_ROUND1)
on configs[1] (92 s clip, full-size synthetic f16 model): prefill logits and 15
greedy decode steps, default (ggml F16C: fp32 fma then fp16) vs round1.
CPU only (test infrastructure); writes a JSON summary."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
import numpy as np
import oracle_py as op
import qasr

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 92.0
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "sens_round1.json")
p = os.environ.get("QASR_FULL_GGUF", "/tmp/qasr_full_f16_s42.gguf")
if not os.path.exists(p):
    qasr.write_synthetic_gguf(p, "full", 42, 1)
op.set_threads(int(os.environ.get("THREADS", os.cpu_count() or 1)))
om = op.OracleModel(p)
pcm = qasr.synth_pcm(16000, int(secs * 16000))   # test_full_configs1_92s's clip
t0 = time.time()
feats = om.encode(op.log_mel(pcm))
ids, pos = om.prompt(feats.shape[0]), 9
print("encode", feats.shape, round(time.time() - t0, 1), "s", flush=True)
res = {}
for name, fl in (("default", 0), ("round1", om.FA_V_ROUND1)):
    t0 = time.time()
    d = op.OracleDecoder(om, len(ids) + steps + 8, fl)
    lg = [d.forward(ids, 0, feats, pos)]
    toks = [int(np.argmax(lg[0]))]
    for k in range(1, steps + 1):
        lg.append(d.forward([toks[-1]], len(ids) + k - 1))
        toks.append(int(np.argmax(lg[-1])))
    res[name] = (lg, toks)
    print(name, round(time.time() - t0, 1), "s", flush=True)
la, ta = res["default"]; lb, tb = res["round1"]
# teacher-forced on the default's tokens as well, so a token flip does not hide the step deltas
d = op.OracleDecoder(om, len(ids) + steps + 8, om.FA_V_ROUND1)
lt = [d.forward(ids, 0, feats, pos)]
for k in range(1, steps + 1):
    lt.append(d.forward([ta[k - 1]], len(ids) + k - 1))
ab = [float(np.abs(x - y).max()) for x, y in zip(la, lt)]
scale = float(np.abs(la[0]).max())
summ = {"secs": secs, "P": len(ids), "steps": steps, "scale": scale, "abs_max": ab, "rel_max": [a / scale for a in ab],
        "greedy_default": ta, "greedy_round1": tb, "greedy_equal": ta == tb,
        "top2_gap_min": float(min(np.sort(x)[-1] - np.sort(x)[-2] for x in la))}
print(json.dumps(summ))
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(summ, open(out, "w"), indent=1)
