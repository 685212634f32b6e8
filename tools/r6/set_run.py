"""The utterance set (configs[3]) alone on one GPU, for A/B runs and profiles:
bench.utterance_set_leg's contexts / slots / queue without the rest of
bench.py.  Env: N_UTT (1000), CTX (2), SLOTS (128), SECS (30), RAGGED=1
(U[5, 30] s lengths from a pool of 256 seeded clips), REPS (1 timed pass after
one warm-up), OPT="name=value,..." (per-context options, qasr_ctx_set_option),
STAGGER_MS (context k starts k x STAGGER_MS late).
Prints one line per pass: RTFx, wall, per-context (clips, refills, steps,
prefill ms, decode ms).  Dev tool (GPU box)."""
import concurrent.futures as cf
import os
import sys
import threading
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
import bench  # noqa: E402
import qasr  # noqa: E402
import qasr_dist as qd  # noqa: E402

# a one-rank RCCL process group, initialised before libqasr.so loads -- bench.py's N > 1 order
if os.environ.get("RCCL") == "1":
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    dist.barrier()

N_UTT = int(os.environ.get("N_UTT", "1000"))
NCTX = int(os.environ.get("CTX", "2"))
# SLOTS: slots per context, one value or one per context ("32,93": asymmetric contexts)
SLOTV = [int(x) for x in os.environ.get("SLOTS", "128").split(",")]
SLOTV = SLOTV * NCTX if len(SLOTV) == 1 else SLOTV
SLOTS = max(SLOTV)
SECS = float(os.environ.get("SECS", "30"))
RAGGED = os.environ.get("RAGGED", "0") == "1"
REPS = int(os.environ.get("REPS", "1"))
OPTS = [kv.split("=") for kv in os.environ.get("OPT", "").split(",") if kv]
STAGGER_MS = float(os.environ.get("STAGGER_MS", "0"))
POOL = 256 if RAGGED else 128

if RAGGED:
    lens = [n for _, n in qd.utterance_set(POOL, 7, 5.0, 30.0)]
else:
    lens = [int(round(SECS * 100)) * 160] * POOL
nmax = max(lens)
bud_max = qd.budget(nmax, 3.5)
P = qasr.lib().qasr_prompt_len(qasr.encoder_frames(qasr.mel_frames(nmax)))
m = qasr.Model(bench.synthetic_model(0))
with cf.ThreadPoolExecutor(16) as ex:
    pcm = list(ex.map(lambda i: qasr.synth_pcm(50000 + i, lens[i]), range(POOL)))
ctxs = [qasr.Context(m, max_batch=SLOTV[k], max_ctx=P + bud_max + 8) for k in range(NCTX)]
for c in ctxs:
    c.stage_audio(pcm)
    c.set_option("staged_wrap", 1)
    for k, v in OPTS:
        c.set_option(k, int(v))
# utterance i = pool clip i % POOL, longest first
order = sorted(range(N_UTT), key=lambda i: -lens[i % POOL])


def run(n_utt):
    lock = threading.Lock()
    nxt = [0]
    todo = [i for i in order if i < n_utt]

    def take():
        with lock:
            if nxt[0] >= len(todo):
                return None
            i = todo[nxt[0]]
            nxt[0] += 1
            return i, qd.budget(lens[i % POOL], 3.5)

    def one(k):
        if STAGGER_MS and k:   # context k starts k x STAGGER_MS late (its refill beside the others' decode)
            time.sleep(k * STAGGER_MS / 1000.0)
        return ctxs[k].run_stream_staged(take, bud_max, ignore_eos=True, slots=SLOTV[k])
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(NCTX) as ex:
        res = list(ex.map(one, range(NCTX)))
    wall = time.perf_counter() - t0
    n = sum(len(o) for o, _ in res)
    assert n == n_utt, n
    audio = sum(lens[i % POOL] for i in range(n_utt)) / 16000.0
    return audio / wall, wall, [(st.n_clips, st.n_prefills, st.n_steps, round(st.t_prefill_ms), round(st.t_decode_ms),
                                 round(st.live_steps / max(1, st.slot_steps), 3)) for _, st in res]


run(min(N_UTT, 2 * sum(SLOTV)))   # warm-up: graphs, buffers
for _ in range(REPS):
    v, wall, st = run(N_UTT)
    print(f"set {N_UTT} x {'U[5,30]' if RAGGED else SECS} s, {NCTX} ctx x {SLOTV} slots, opts {OPTS}, stagger {STAGGER_MS} ms: "
          f"{v:.1f} RTFx  wall {wall:.3f} s  "
          f"per ctx (clips, refills, steps, prefill ms, decode ms, slot util) {st}", flush=True)
for c in ctxs:
    c.close()
