"""Experiment: the utterance set through several continuous-batching contexts at
once on one GPU (each its own HIP stream, driven by its own host thread from
one shared queue), so one context's refill prefill can overlap another's
decode steps.  Prints RTFx per (contexts x slots).  Dev tool (GPU box)."""
import os
import sys
import threading
import time
import concurrent.futures as cf

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "qwen3-asr.cpp_amd", "python"))
import bench  # noqa: E402
import qasr  # noqa: E402
import qasr_dist as qd  # noqa: E402

N_UTT, SECS, POOL = int(os.environ.get("N_UTT", "1000")), 30.0, 128
ns = int(round(SECS * 100)) * 160
bud = qd.budget(ns, 3.5)
P = qasr.lib().qasr_prompt_len(qasr.encoder_frames(qasr.mel_frames(ns)))
m = qasr.Model(bench.synthetic_model(0))
with cf.ThreadPoolExecutor(16) as ex:
    pcm = list(ex.map(lambda i: qasr.synth_pcm(50000 + i, ns), range(POOL)))


def run(nctx: int, slots: int, n_utt: int, stagger_s: float = 0.0):
    ctxs = [qasr.Context(m, max_batch=slots, max_ctx=P + bud + 8) for _ in range(nctx)]
    for c in ctxs:
        c.stage_audio(pcm)
        c.set_option("staged_wrap", 1)
    lock = threading.Lock()
    nxt = [0]

    def next_clip():
        with lock:
            if nxt[0] >= n_utt:
                return None
            i = nxt[0]
            nxt[0] += 1
            return i

    def one(k_c):
        k, c = k_c
        if k and stagger_s > 0:
            time.sleep(k * stagger_s)   # context k starts k staggers late: refills alternate with the others' decode
        out, st = c.run_stream_staged(next_clip, bud, ignore_eos=True, slots=slots)
        return out, st
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(nctx) as ex:
        res = list(ex.map(one, list(enumerate(ctxs))))
    wall = time.perf_counter() - t0
    n = sum(len(o) for o, _ in res)
    for c in ctxs:
        c.close()
    assert n == n_utt, n
    toks = {}
    for o, _ in res:
        toks.update(o)
    return n_utt * SECS / wall, [(st.n_prefills, round(st.t_prefill_ms), round(st.t_decode_ms)) for _, st in res], toks


ref = None
for nctx, slots, stg in [(1, 128, 0.0), (2, 128, 0.0), (2, 128, 0.2), (2, 128, 0.35), (2, 128, 0.5), (3, 128, 0.0), (3, 128, 0.15)]:
    run(nctx, slots, min(N_UTT, 2 * nctx * slots))   # warm-up (graphs, buffers)
    v, st, toks = run(nctx, slots, N_UTT, stg)
    if ref is None:
        ref = toks
    same = all(toks[i] == ref[i] for i in ref)
    print(f"{nctx} ctx x {slots} slots, stagger {stg} s: {v:.1f} RTFx  tokens equal to 1 x 128: {same}  per ctx (refills, "
          f"prefill ms, decode ms) {st}", flush=True)
