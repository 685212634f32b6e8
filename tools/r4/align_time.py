"""configs[4]'s aligner leg on one 92 s clip: wall time of qasr_align_json_batch
against its own stage timings (mel / encode / prefill+classify / total)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
import bench  # noqa: E402
import qasr  # noqa: E402

m = qasr.Model(bench.synthetic_model(0, "full", 1))
n = 92 * 16000
pcm = qasr.synth_pcm(1000, n)
c = qasr.Context(m, max_batch=1, max_ctx=1600)
toks = c.transcribe([pcm], max_tokens=322, ignore_eos=True).tokens[0]
text = m.detokenize(toks)
am = qasr.Model(bench.synthetic_model(0, "aligner", 1))
need = qasr.align_prompt_len(n, len(am.align_tokenize(text)[0]))
ac = qasr.Context(am, max_batch=1, max_ctx=need + 8)
print("words", len(text.split()), "prompt", need, flush=True)
for it in range(4):
    t0 = time.perf_counter()
    docs, t = ac.align_json_batch([pcm], [text])
    dt = (time.perf_counter() - t0) * 1e3
    print(f"wall {dt:.2f} ms  mel {t.t_mel_ms:.2f} enc {t.t_encode_ms:.2f} prefill {t.t_prefill_ms:.2f} "
          f"decode {t.t_decode_ms:.2f} total {t.t_total_ms:.2f}", flush=True)
