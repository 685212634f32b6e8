#!/usr/bin/env python3
"""bench.py -- RTFx + decode tok/s of the MI355X-native Qwen3-ASR hot path.

Metric (BASELINE.json): RTFx (audio-sec / wall-sec) + decode tokens/s,
Qwen3-ASR-0.6B f16.  A "step" = one full transcription (mel -> conv front-end
-> encoder -> prompt splice -> prefill -> greedy decode) of the configs[1]
workload per GPU: one 92 s / 16 kHz clip (the README benchmark clip length,
README.md:129-138; synthetic audio since the Korean WAV is not shipped) with
the fixed decode budget ceil(3.5 tok/s x 92 s) = 322 tokens, EOS ignored
(SURVEY.md §8(d)).  Weights: synthetic Qwen3-ASR-0.6B-shaped f16 GGUF
(random init, reference tensor names/shapes) unless $QASR_MODEL is set.
PCM is staged in HBM before the timed region (qasr_stage_audio).

Multi-GPU: one process per GPU (torchrun); each rank transcribes its own clips
(weak scaling, no data-path collective); barrier + max-over-ranks timing via
torch.distributed (RCCL); value = all ranks' audio-seconds / max wall time.
"""
import argparse
import json
import math
import os
import sys
import time

# HIP hardware queues per process (HIP's default, 4 on the GPU box): the utterance set's
# context streams, the default stream and RCCL's share queues beyond that -- with 8, three
# contexts 9360-9375 -> 9626-9690 RTFx and four 9986-10031 (profiles/r6/hw_queues.txt).  The
# HIP runtime reads it at its first call: set before anything below touches the GPU.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import qasr  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
README_RTFX = 92.0 / 5.007   # 92 s clip in 5,007 ms on M2 Pro (README.md:136)
README_ALIGN_RTFX = 92.0 / 18.005   # transcribe + align of the same clip (README.md:138)
MFMA_F16_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense fp16 MFMA (no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node; without a launcher (WORLD_SIZE unset) N > 1 spawns one rank per GPU")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=92.0, help="clip length (configs[1]: 92 s)")
    ap.add_argument("--batch", type=int, default=1, help="clips per GPU per step")
    ap.add_argument("--tok-rate", type=float, default=3.5, help="decode budget tokens per audio second")
    ap.add_argument("--model", default=os.environ.get("QASR_MODEL", ""))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-seconds", type=float, default=10.0)
    ap.add_argument("--probe-layer", type=int, default=14, help="decoder layer whose fused launches are probed")
    ap.add_argument("--fa-exact-decode", type=int, default=None, choices=(0, 1),
                    help="decode attention numerics: 1 = ggml's fp16 V accumulation (the engine default; batch 1 f16: the "
                         "fused launch's chain role), 0 = fp32 accumulation (split-K)")
    ap.add_argument("--cpu-threads", type=int, default=4, help="reference's effective ggml thread count")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--probe-stride", type=int, default=8, help="probe every k-th decode step (roofline)")
    ap.add_argument("--q8", action="store_true", help="Q8_0 synthetic model (configs[2] weights)")
    ap.add_argument("--pipeline", choices=("asr", "align"), default="asr",
                    help="align: configs[4] transcribe + ForcedAligner on every clip (src/main.cpp:416-500)")
    ap.add_argument("--queue", choices=("dynamic", "static"), default="dynamic",
                    help="--utterances: a shared work queue feeding each GPU's continuous-batching stream (dynamic), "
                         "or the static longest-first shards in fixed batches (static)")
    ap.add_argument("--utterances", type=int, default=0,
                    help="configs[3]/[4]: a fixed set of N seeded utterances of U[--utt-min, --utt-max] s sharded "
                         "longest-first over the ranks (strong scaling); a step = one pass over the set")
    ap.add_argument("--utt-min", type=float, default=5.0)
    ap.add_argument("--utt-max", type=float, default=30.0)
    ap.add_argument("--utt-seed", type=int, default=0)
    ap.add_argument("--align-batch", type=int, default=32,
                    help="--pipeline align: clips per ForcedAligner pass (qasr_align_json_batch)")
    ap.add_argument("--dump-align", default="",
                    help="--pipeline align with --utterances: rank 0 writes its shortest utterance's id, transcript and "
                         "aligner document from the last timed pass to this JSON file (tests/test_gpu_api.py checks it "
                         "against the oracle)")
    ap.add_argument("--set-utterances", type=int, default=1000,
                    help="the default run's utterance_set leg (configs[3], SURVEY.md §8(d)): N fixed-length utterances "
                         "through the dynamic queue into each GPU's continuous-batching stream, strong scaling over the "
                         "ranks (0: skip)")
    ap.add_argument("--set-seconds", type=float, default=30.0)
    ap.add_argument("--set-pool", type=int, default=128, help="distinct seeded clips staged per GPU (utterance i = clip i mod pool)")
    ap.add_argument("--set-slots", type=int, default=128, help="continuous-batching slots per context")
    ap.add_argument("--set-contexts", type=int, default=0,
                    help="continuous-batching contexts per GPU, each on its own HIP stream and host thread, all fed by "
                         "the rank's queue (one context's refill prefill overlaps another's decode steps); 0 = by the "
                         "rank's share of the set (set_contexts)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous check without a GPU: ranks join a gloo group, time a barrier and rank 0 "
                         "prints the JSON line with value 0 (tests/test_dist.py)")
    return ap.parse_args()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): spawn N child
    processes of this same command, one per GPU, with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (what torch.distributed.run
    would set), wait for all of them and return the first non-zero exit code.
    This parent never touches the GPU (no HIP call, no torch import), so the
    children are plain forks + execs of a GPU-free process.  Rank 0 prints the
    JSON line; the others print nothing on stdout."""
    import signal
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    for q in procs:   # one rank failed: the others would wait in a collective forever
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def dry_run(args, world: int, rank: int) -> None:
    """The launcher's rendezvous without the GPU: gloo group, barrier-timed
    region, max over ranks, rank 0's line."""
    if os.environ.get("QASR_BENCH_FAIL_RANK") == str(rank):   # (the launcher test's failing rank)
        sys.exit(3)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "audio-sec/wall-sec", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f16",
                          "data": "none (dry run)", "config": {"workload": "dry run", "parallelism": f"dp{world}"}}),
              flush=True)
    if dist is not None:
        dist.destroy_process_group()


def synthetic_model(rank: int, config: str = "full", wtype: int = 1, seed: int = 42) -> str:
    """The synthetic GGUF, written once per host by rank 0 and shared.  The
    cache is keyed on everything the file depends on -- config, weight type,
    seed and the writer's output version (qasr_synthetic_gguf_version) -- and
    the marker records the file's size, so neither a file of an older writer
    nor a torn write is ever reused."""
    ver = int(qasr.lib().qasr_synthetic_gguf_version())
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"),
                        f"qasr_synth_{config}_{'q8_0' if wtype == 8 else 'f16'}_s{seed}_w{ver}.gguf")
    lock = path + ".done"

    def valid():
        try:
            return os.path.exists(path) and int(open(lock).read().strip()) == os.path.getsize(path)
        except (OSError, ValueError):
            return False
    if rank == 0 and not valid():
        qasr.write_synthetic_gguf(path + ".tmp", config, seed, wtype)
        os.replace(path + ".tmp", path)
        with open(lock + ".tmp", "w") as f:
            f.write(str(os.path.getsize(path)))
        os.replace(lock + ".tmp", lock)
    while not valid():
        time.sleep(0.5)
    return path


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(model_path: str, secs: float, tok_rate: float, threads: int, full_secs: float, full_tok: int):
    """Oracle (C restatement of the reference CPU path, ggml numerics) timed
    on configs[0]'s own workload -- one 30 s clip, its 105-token budget, no
    extrapolation -- at the reference's effective thread count (4: ggml's
    default; mel single-threaded as the reference) and at
    every core this process may use (the GPU box's lease: OMP_NUM_THREADS),
    plus the shorter `secs` sample with its per-stage extrapolation to the
    bench's own clip (configs[1])."""
    import oracle_py as op
    om = op.OracleModel(model_path)
    allc = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 10 ** 6))

    def timed(clip_s, th):
        n = int(clip_s * 16000)
        ntok = int(math.ceil(tok_rate * clip_s))
        op.set_threads(th)
        t0 = time.perf_counter()
        _, t = om.transcribe(qasr.synth_pcm(1000, n), max_tokens=ntok, ignore_eos=True)
        dt = time.perf_counter() - t0
        return dt, t, ntok

    c0 = {}   # configs[0]: 30 s, measured
    for th in sorted({threads, allc}):
        dt, t, ntok = timed(30.0, th)
        c0[th] = {"rtfx": round(30.0 / dt, 4), "wall_s": round(dt, 3), "tokens": ntok,
                  "stage_ms": {"mel": round(t[0], 1), "encode+prefill": round(t[1], 1), "decode": round(t[2], 1)}}
    runs = {}   # the short sample, extrapolated per stage to the bench clip
    for th in sorted({threads, allc}):
        dt, t, ntok = timed(secs, th)
        est = (t[0] + t[1]) / 1e3 * (full_secs / secs) + t[2] / 1e3 * (full_tok / ntok)
        runs[th] = {"rtfx": round(secs / dt, 4), "wall_s": round(dt, 3),
                    "stage_ms": {"mel": round(t[0], 1), "encode+prefill": round(t[1], 1), "decode": round(t[2], 1)},
                    "est_configs1_rtfx": round(full_secs / est, 4)}
    r4 = c0[threads]
    return {
        "value": r4["rtfx"],
        "unit": "audio-sec/wall-sec (RTFx)",
        "cores": threads,
        "kind": "port",
        "sample": f"configs[0] measured at its own size: one 30 s synthetic clip, {r4['tokens']}-token greedy budget, "
                  f"full-size synthetic f16 model, {threads} threads (ggml's default; mel single-thread fp64 DFT as the "
                  f"reference); at all {allc} leased cores {c0[allc]['rtfx']} RTFx.  The {secs:g} s sample extrapolated "
                  f"to the bench clip ({full_secs:g} s, {full_tok} tokens): {runs[threads]['est_configs1_rtfx']} RTFx",
        "configs0_by_threads": c0,
        "runs_by_threads": runs,
        "all_cores": allc,
        "nproc": os.cpu_count(),
        "cpu_model": cpu_model(),
    }


ATTN_LABEL = {
    0: "fp32 V accumulation (split-K)",
    1: "fp16 V accumulation per key (ggml CPU flash-attention numerics; chain role of the fused QKV + attention + "
       "o-proj launch)",
    2: "fp16 V accumulation per key (ggml CPU flash-attention numerics; scores + chain in one launch per kv group and "
       "sequence, decode_attn_seq_kernel)",
    3: "fp16 V accumulation per key (ggml CPU flash-attention numerics; separate scores + chain kernels)",
}


def pmc_traffic(kernel_prefix: str):
    """HBM bytes per launch of the roofline kernel from the newest committed
    rocprofv3 PMC summary (profiles/<round>/summary.json, tools/profile_round.sh:
    separate FETCH_SIZE / WRITE_SIZE passes, gfx950 FETCH x2 correction)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k in d.get("kernels", []):
            if k["name"].startswith(kernel_prefix) and "hbm_read_bytes" in k:
                return k["hbm_read_bytes"] + k.get("hbm_write_bytes", 0), os.path.relpath(f, ROOT)
    return None, None


def pmc_group_traffic(kind: int, batch: int, q8: bool):
    """HBM bytes of one probed batch launch group (kind 2: QKV projection +
    attention; kind 3: o-proj + FFN) from the newest committed batch PMC
    summary (profiles/<round>/batch/{f16,q8}/summary.json, tools/profile_batch.sh)
    whose bench line ran this batch size.  Per layer-step: the attention
    kernel's calls count the layer-steps; the QKV skinny GEMM is the plain-epilogue
    instance launched once per layer-step, the SwiGLU instance and the o/down
    instance go to the FFN group.  The rmsnorm launches are left out: their
    profile line mixes the prefill's 64 x P-row launches with the decode's
    64-row ones (0.4 MB a launch, under 0.5 % of either group)."""
    import glob
    import re
    sub = "q8" if q8 else "f16"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "batch", sub, "summary.json")), reverse=True):
        try:
            d = json.load(open(f))
            bl = json.load(open(os.path.join(os.path.dirname(f), "bench.json")))
        except (OSError, ValueError):
            continue
        if bl.get("config", {}).get("clips_per_gpu") != batch:
            continue
        ks = [k for k in d.get("kernels", []) if "hbm_read_bytes" in k]
        att = [k for k in ks if k["name"].startswith("void qasr::decode_attn")]
        if not att:
            continue
        ls = max(k["calls"] for k in att)
        tot = {2: 0.0, 3: 0.0}
        for k in ks:
            per = (k["hbm_read_bytes"] + k.get("hbm_write_bytes", 0)) * k["calls"] / ls
            n = k["name"]
            if n.startswith("void qasr::decode_attn"):
                tot[2] += per
            elif n.startswith("void qasr::gemm_skinny"):
                m = re.match(r"void qasr::gemm_skinny\w*<([^>]*)>", n)
                epi = int(m.group(1).split(",")[3]) if m else 0
                tot[2 if epi == 0 and k["calls"] == ls else 3] += per
        return round(tot[kind]), os.path.relpath(f, ROOT)
    return None, None


def profiled_mfma():
    """Time-weighted MFMA utilisation of the encoder / prefill MFMA kernels
    from the newest committed rocprofv3 MFMA-counter pass (tools/prof_report.py)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ks = [k for k in d.get("kernels", []) if "mfma_util" in k]
        if not ks:
            continue
        t = sum(k["total_ms"] for k in ks)
        top = max(ks, key=lambda k: k["total_ms"])
        return {"mfma_util": round(sum(k["mfma_util"] * k["total_ms"] for k in ks) / t, 4), "kernels": len(ks),
                "kernel_ms": round(t, 3), "top_kernel": top["name"][:96], "top_mfma_util": top["mfma_util"],
                "top_mfma_tflops": top.get("mfma_tflops"), "source": os.path.relpath(f, ROOT)}
    return None


def roofline_entry(kind: int, batch: int, total_ms: float, n: int, bytes_per_launch: float, dev_ms: float, dev_n: int,
                   layer: int, exact: bool = False, q8: bool = False) -> dict:
    """HBM roofline of one probed launch group: algorithmic bytes per launch
    (engine.hip probe_bytes: weights + the layer's K/V rows at each step's
    n_kv, averaged over the probed steps) / its mean duration.  Both clocks of
    the same launches in the timed region: HIP events on the context stream
    around the launch (includes ~2.5 us of dispatch + event processing), and
    the device clock folded in-kernel (first workgroup start -> last
    workgroup end: what rocprofv3 --kernel-trace reports as the kernel's
    duration).  achieved / frac use the device clock where it exists."""
    ev_s = total_ms / n / 1e3
    avg_s = dev_ms / dev_n / 1e3 if dev_n else ev_s
    achieved = bytes_per_launch / avg_s / 1e9
    b1 = batch == 1
    if kind == 2 and exact:
        kname = ("qkv_attn1_kernel (batch 1: rmsnorm + QKV GEMV + attention scores + ggml fp16-V chain + o-proj, one launch)"
                 if b1 else "decode layer QKV projection + exact attention (kernel group)")
        prefix = "void qasr::qkv_attn1_kernel<" if b1 else None
    elif kind == 2:
        kname = ("qkv_attn1_kernel (batch 1: rmsnorm + QKV GEMV + split-K attention + o-proj, one launch)" if b1 else
                 "decode layer QKV projection + attention (kernel group)")
        prefix = "void qasr::qkv_attn1_kernel<" if b1 else None
    elif kind == 3:
        kname = "ffn1_kernel (batch 1: rmsnorm + gate/up SwiGLU + down + residual, one launch)" if b1 else \
            "decode layer FFN (kernel group)"
        prefix = "void qasr::ffn1_kernel<" if b1 else None
    else:
        kname = "LM head (tied 151936x1024 f16 GEMV + fused argmax)"
        prefix = f"void qasr::gemv_kernel<3, 4, {next(r for r in (1, 2, 4, 8) if r >= batch)}," if batch <= 8 else None
    if prefix:
        traffic, src = pmc_traffic(prefix)
    elif kind in (2, 3):
        traffic, src = pmc_group_traffic(kind, batch, q8)
    else:
        traffic, src = None, None
    return {"kernel": kname + (f", decoder layer {layer}" if kind != 1 else ""), "bound": "hbm",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "traffic_source": src, "bytes_per_launch": round(bytes_per_launch),
            "avg_launch_us": round(avg_s * 1e6, 2), "clock": "device" if dev_n else "hip_events",
            "avg_launch_us_hip_events": round(ev_s * 1e6, 2), "launches": n,
            "frac_hip_events": round(bytes_per_launch / ev_s / 1e9 / HBM_PEAK_GBS, 4)}


def encoder_flops(hp, n_samples: int) -> float:
    """Algorithmic FLOPs of the ASR audio encoder for one clip (SURVEY.md §8(d):
    278.0 GFLOP per 30 s): conv front-end per 100-frame chunk (3x3 s2 convs,
    conv_out), full-attention transformer over all frames, post projections."""
    T = qasr.mel_frames(n_samples)
    C, D, F, L = hp.conv_channels, hp.d_model, hp.enc_ffn, hp.enc_layers
    o = lambda w: (w - 1) // 2 + 1
    mac, N = 0, 0
    for c0 in range(0, T, 100):
        w1 = o(min(100, T - c0)); w2 = o(w1); w3 = o(w2)
        mac += 64 * w1 * C * 9 + 32 * w2 * C * 9 * C + 16 * w3 * C * 9 * C + w3 * 16 * C * D
        N += w3
    mac += L * (4 * N * D * D + 2 * N * D * F + 2 * N * N * D) + N * D * (D + hp.hidden_size)
    return 2.0 * mac


def decode_bytes(hp, q8: bool, batch: int, prompt: int, ntok: int) -> float:
    """Algorithmic HBM bytes of the decode loop: every step
    streams the decoder weights once (shared by the batch) plus each sequence's
    K/V cache rows 0..n_kv-1 (fp16, all layers)."""
    H, hd = hp.hidden_size, hp.head_dim
    per_layer = (hp.n_heads * hd + 2 * hp.n_kv_heads * hd) * H + H * hp.n_heads * hd + 3 * hp.dec_ffn * H
    w = hp.dec_layers * per_layer * (34 / 32 if q8 else 2) + hp.vocab_size * H * 2
    kv_row = hp.dec_layers * 2 * hp.n_kv_heads * hd * 2
    kv = sum(kv_row * (prompt + s + 1) for s in range(ntok))
    return ntok * w + batch * kv


def workload(args, ntok: int, align: bool) -> str:
    """the BASELINE.json config this run is (configs[1] by default)"""
    if align:
        name = "configs[4]: transcribe + ForcedAligner"
    elif args.q8 and args.batch > 1:
        name = "configs[2]: q8_0 batch"
    elif args.batch == 1 and not args.q8 and args.seconds == 92.0:
        name = "configs[1]"
    else:
        name = "custom"
    return (f"{name}: {args.batch} x {args.seconds:g} s clip(s) per GPU per step, greedy decode budget {ntok} tokens "
            f"(3.5 tok/s), EOS ignored")


def utterance_main(args, m, rank, local, world, dist, model_path):
    """configs[3] (and [4] with --pipeline align): the sharded driver of
    qasr_dist.run_shard over a fixed utterance set; each rank stages its whole
    shard in HBM before the timed region and runs it in batches from there."""
    import qasr_dist as qd
    utts = qd.utterance_set(args.utterances, args.utt_seed, args.utt_min, args.utt_max)
    lengths = [n for _, n in utts]
    batch = args.batch if args.batch > 1 else 64
    dynamic = args.queue == "dynamic"
    # dynamic: any rank may take any utterance, so every rank stages them all
    shard = list(range(len(utts))) if dynamic else qd.shard_longest_first(lengths, world)[rank]
    nmax = max(lengths)
    P = qasr.lib().qasr_prompt_len(qasr.encoder_frames(qasr.mel_frames(nmax)))
    ctx = qasr.Context(m, max_batch=batch, max_ctx=P + qd.budget(nmax, args.tok_rate) + 8)
    pcm = {i: qasr.synth_pcm(utts[i][0], utts[i][1]) for i in shard}
    pos = {i: k for k, i in enumerate(shard)}
    if shard:
        ctx.stage_audio([pcm[i] for i in shard])

    def transcribe(idx, max_tokens):
        return ctx.run_staged([pos[i] for i in idx], max_tokens, ignore_eos=True).tokens

    stream_stats = []

    def stream(next_clip):   # staged index = utterance index (all staged, in order)
        out, st = ctx.run_stream_staged(next_clip, max(qd.budget(n, args.tok_rate) for n in lengths), ignore_eos=True)
        bad = [i for i, t in out.items() if isinstance(t, Exception)]
        assert not bad, (bad[:4], out[bad[0]] if bad else None)
        stream_stats.append(st)
        return out

    passes = [0]

    def one_pass(after):
        passes[0] += 1
        if dynamic:
            return qd.run_queue(stream, utts, rank, world, args.tok_rate, dist, f"cuda:{local}" if dist else None,
                                key=f"utt_queue_{passes[0]}", after=after)
        return qd.run_shard(transcribe, utts, rank, world, batch, args.tok_rate, dist, f"cuda:{local}" if dist else None,
                            after)

    after = None
    actx = None
    aligned = set()
    kept = {}   # --dump-align: rank 0's shortest utterance -> (transcript, document) of the latest pass
    keep = min(shard, key=lambda i: utts[i][1]) if shard and args.dump_align and rank == 0 else None
    if args.pipeline == "align":   # configs[4]: ForcedAligner on every transcript (src/main.cpp:416-500)
        am_path = os.environ.get("QASR_ALIGNER_MODEL") or synthetic_model(rank, "aligner", 8 if args.q8 else 1)
        am = qasr.Model(am_path, local)
        # prompt: audio pads + per word its BPE ids and two timestamps (ForcedAligner::tokenize_with_timestamps)
        ab = args.align_batch
        actx = qasr.Context(am, max_batch=ab, max_ctx=P + 8 * qd.budget(nmax, args.tok_rate) + 64)

        def after(idx, toks):   # the rank's transcripts, ab clips per aligner pass (qasr_align_json_batch)
            for k in range(0, len(idx), ab):
                sub = idx[k:k + ab]
                texts = [m.detokenize(t) for t in toks[k:k + ab]]
                docs, _ = actx.align_json_batch([pcm[i] for i in sub], texts)
                assert len(docs) == len(sub) and all(isinstance(d, dict) for d in docs), sub
                aligned.update(sub)
                if keep in sub:
                    kept[keep] = (texts[sub.index(keep)], docs[sub.index(keep)])
    for _ in range(args.warmup):
        one_pass(after)
    wall, res = 0.0, None
    stream_stats.clear()
    for _ in range(args.steps):
        res = one_pass(after)
        wall += res["wall_s"]
    if rank != 0:
        return
    toks = res["tokens"]
    assert len(toks) == len(utts), (len(toks), len(utts))
    assert all(len(toks[i]) == qd.budget(n, args.tok_rate) for i, (_, n) in enumerate(utts)), "decode budget not met"
    audio = res["audio_s"] * args.steps
    out = {
        "metric": "RTFx (audio-sec/wall-sec) + decode tokens/sec, Qwen3-ASR-0.6B " + ("q8_0" if args.q8 else "f16") +
                  (" + ForcedAligner-0.6B (transcribe-align)" if actx else ""),
        "value": round(audio / wall, 3),
        "unit": "audio-sec/wall-sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "q8_0 weights, int8 x int8 -> fp32" if args.q8 else "f16",
        "data": "synthetic (seeded 16 kHz clips; random-init Qwen3-ASR-0.6B-shaped GGUF"
                + (", ForcedAligner-0.6B-shaped aligner GGUF)" if actx else ")"),
        "config": {"workload": f"{'configs[4]' if actx else 'configs[3]'}: {len(utts)} utterances of "
                               f"U[{args.utt_min:g}, {args.utt_max:g}] s (seed {args.utt_seed}, {res['audio_s']:.0f} s of "
                               f"audio) over {world} GPU(s), "
                               + (f"a shared longest-first queue feeding {batch} continuous-batching slots per GPU"
                                  if dynamic else f"sharded longest-first, batches of {batch} per GPU")
                               + ", greedy budget ceil(3.5 tok/s x duration), EOS ignored",
                   "utterances": len(utts), "batch_per_gpu": batch, "queue": args.queue,
                   "parallelism": f"dp{world} (utterance data parallelism)",
                   "collectives": "barrier + max wall time + one all_gather of token ids (RCCL), none on the data path"
                                  + ("; the queue is a TCPStore counter (one add per utterance)" if dynamic and world > 1
                                     else "")},
        "decode_tokens_per_s": round(res["decode_tokens"] * args.steps / wall, 2),
    }
    if actx is not None:
        out["aligned_rank0"] = len(aligned)
        if keep is not None:
            assert keep in kept, "the kept utterance was not aligned on rank 0"
            # (untimed) the same clip's raw timestamp classes, single-clip: the test checks the document against them
            # and them against the oracle
            cls, _ = actx.align(pcm[keep], am.align_tokenize(kept[keep][0])[0])
            with open(args.dump_align, "w") as f:
                json.dump({"utterance": keep, "seed": utts[keep][0], "n_samples": utts[keep][1], "text": kept[keep][0],
                           "doc": kept[keep][1], "classes": [int(x) for x in cls], "aligner_model": am_path,
                           "asr_model": model_path}, f)
    if dynamic:
        ss = stream_stats
        out["rank0_stream"] = {"clips": sum(x.n_clips for x in ss), "refill_prefills": sum(x.n_prefills for x in ss),
                               "decode_steps": sum(x.n_steps for x in ss),
                               "slot_utilisation": round(sum(x.live_steps for x in ss) / max(1, sum(x.slot_steps for x in ss)), 4),
                               "prefill_ms": round(sum(x.t_prefill_ms for x in ss), 1),
                               "decode_ms": round(sum(x.t_decode_ms for x in ss), 1)}
    else:
        out["batches_per_rank0_pass"] = res["batches"]
    print(json.dumps(out), flush=True)


def pmc_batch_kernel(kernel_prefix: str, batch: int, sub: str = "f16"):
    """HBM bytes per launch of one decode-batch kernel from the newest committed
    single-context batch PMC summary (profiles/<round>/batch*/<sub>/summary.json,
    tools/profile_batch.sh) whose bench line ran this batch size"""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "batch*", sub, "summary.json")), reverse=True):
        try:
            d = json.load(open(f))
            bl = json.load(open(os.path.join(os.path.dirname(f), "bench.json")))
        except (OSError, ValueError):
            continue
        if bl.get("config", {}).get("clips_per_gpu") != batch:
            continue
        for k in d.get("kernels", []):
            if k["name"].startswith(kernel_prefix) and "hbm_read_bytes" in k:
                return k["hbm_read_bytes"] + k.get("hbm_write_bytes", 0), os.path.relpath(f, ROOT)
    return None, None


def set_decode_bytes(hp, stats) -> float:
    """Algorithmic HBM bytes of the contexts' decode steps: per
    step the decoder weights and the tied LM head once (shared by the slots),
    plus every slot's K / V cache rows 0..n_kv-1 (qasr_stream_stats.kv_keys)"""
    H, hd = hp.hidden_size, hp.head_dim
    per_layer = (hp.n_heads * hd + 2 * hp.n_kv_heads * hd) * H + H * hp.n_heads * hd + 3 * hp.dec_ffn * H
    w = hp.dec_layers * per_layer * 2 + hp.vocab_size * H * 2
    kv_row = hp.dec_layers * 2 * hp.n_kv_heads * hd * 2
    return float(sum(st.n_steps * w + st.kv_keys * kv_row for st in stats))


def set_contexts(share: int, slots: int = 128) -> int:
    """Contexts per GPU for a rank's share of the utterance set (round 6,
    tools/r6/set_run.py on one MI355X, RTFx; profiles/r6/set_contexts.txt,
    profiles/r6/set_contexts_r6b.txt): 125 utterances (N = 8) 1 x 125 slots
    7849, 2 x 63 7603, 3 x 42 7369 -- every context's decode step costs about
    a full-width step, so splitting a small share only adds steps (asymmetric
    splits 32 + 93 etc.: 7295-7546; two 63-slot contexts started 60-140 ms
    apart: 7407-7784 against 8259 for one); 250: 2 x 125 8721, 3 x 84 8343;
    500: 2 x 128 8688, 3 x 128 8736.  1000, after the round-6 kernels: three
    contexts of 128 slots 9322-9558 against two 9276-9356 (set_run.py, four
    runs each), 9343-9601 against 9279-9280 in the bench line, and the ragged
    set 9753-9828 against 9387-9473 -- a third context's refill fills more of
    the other two's decode gaps.  With 8 hardware queues a process
    (GPU_MAX_HW_QUEUES, set at the top of this file; HIP's default 4 made
    streams share queues): three contexts 9626-9690, four 9986-10031, the
    ragged set 9802-9841 / 10078-10205 (profiles/r6/hw_queues.txt); five
    9690-9776, six (16 queues) 9370-9399; a 500-utterance share (N = 2) four
    contexts 9936-9950 against three 8492-9362 (profiles/r6/
    set_contexts_hwq8.txt).  So: one context for a share that fits one, two
    for up to two contexts' slots, four beyond."""
    return 1 if share <= slots else 2 if share <= 2 * slots else 4


def utterance_set_leg(args, m, rank, local, world, dist) -> dict:
    """configs[3] inside the default run (1000 x 30 s f16
    utterances; north_star's "throughput on synthetic 30 s / 16 kHz audio at
    1, 2, 4 and 8 GPUs"): every rank stages a pool of distinct seeded 30 s
    clips in HBM (utterance i = pool clip i mod pool; the engine processes each
    utterance in full -- nothing is cached across them), then one shared
    longest-first queue in the process group's TCPStore feeds each rank's
    continuous-batching stream (qasr_run_stream_staged, --set-slots slots):
    strong scaling, the set is fixed whatever N is.  One warm-up pass over a
    subset (graph capture), then one timed pass: barrier -> streams -> barrier,
    wall = max over ranks; each rank's own stream time and utterance count are
    gathered for the tail imbalance.  Budget ceil(3.5 tok/s x 30 s) = 105
    tokens a clip, EOS ignored (every budget is asserted).  Each rank runs
    --set-contexts contexts of --set-slots slots concurrently (own HIP stream,
    own host thread, one lock around the rank's queue): a context's refill
    prefill (compute-bound) overlaps the others' decode steps (latency / HBM
    bound) -- 1 x 128 slots 7780, 2 x 128 8500, 3 x 128 8690 RTFx, tokens equal
    (tools/r5/two_ctx.py; 4 contexts exceed the box's 4 hardware queues).
    Round 6: the set's own rooflines from one untimed
    single-context pass after the timed one (so the contexts do not contend):
    the dominant decode kernel (decode_attn_seq_kernel<1>, layer probe_layer,
    device clock) and the encoder by its HIP events; the timed pass's decode
    bytes (weights + every slot's K / V rows) over the contexts' decode time;
    and SURVEY.md §8(d)'s ragged form: --set-utterances x U[5, 30] s with
    natural-length budgets through the same queue (`ragged`)."""
    import concurrent.futures as cf
    import threading

    import qasr_dist as qd
    n_utt, secs = args.set_utterances, args.set_seconds
    ns = int(round(secs * 100)) * 160
    utts = [(50000 + i, ns) for i in range(n_utt)]
    bud = qd.budget(ns, args.tok_rate)
    P = qasr.lib().qasr_prompt_len(qasr.encoder_frames(qasr.mel_frames(ns)))
    nctx = args.set_contexts if args.set_contexts > 0 else set_contexts(-(-n_utt // world), args.set_slots)
    # slots per context: --set-slots, or fewer when the rank's share of the set cannot fill them
    # (strong scaling: 1000 utterances over 8 ranks x 2 contexts is ~63 a context; parked slots
    # would still cost a decode step its full-batch GEMMs)
    slots = max(1, min(args.set_slots, -(-n_utt // (world * nctx))))
    ctxs = [qasr.Context(m, max_batch=slots, max_ctx=P + bud + 8) for _ in range(nctx)]
    pool = min(args.set_pool, n_utt)
    with cf.ThreadPoolExecutor(16) as ex:   # (ctypes releases the GIL: the C synthesiser runs in parallel)
        pcm = list(ex.map(lambda i: qasr.synth_pcm(utts[i][0], ns), range(pool)))
    for c in ctxs:
        c.stage_audio(pcm)
        c.set_option("staged_wrap", 1)   # utterance ids past the pool reuse its clips (id % pool)
    stats = []

    def stream(next_clip):
        lock = threading.Lock()

        def take():   # the rank's queue (a TCPStore client) is not shared between threads unguarded
            with lock:
                return next_clip()

        def one(c):
            out, st = c.run_stream_staged(take, bud, ignore_eos=True, slots=slots)
            bad = [i for i, t in out.items() if isinstance(t, Exception)]
            assert not bad, (bad[:4], out[bad[0]] if bad else None)
            return out, st
        with cf.ThreadPoolExecutor(nctx) as ex:
            res = list(ex.map(one, ctxs))
        merged = {}
        for out, st in res:
            merged.update(out)
            stats.append(st)
        return merged
    dev = f"cuda:{local}" if dist else None
    warm = utts[:min(n_utt, 2 * slots * nctx * world)]
    qd.run_queue(stream, warm, rank, world, args.tok_rate, dist, dev, key="utt_set_warm")
    stats.clear()
    res = qd.run_queue(stream, utts, rank, world, args.tok_rate, dist, dev, key="utt_set_timed")
    timed = list(stats)

    # the set's rooflines (untimed, one context alone): one staged refill of `slots` clips at the
    # set's shape through qasr_run_staged, the layer's attention launch probed by the device clock
    c0 = ctxs[0]
    c0.set_option("probe_layer", args.probe_layer)
    c0.set_option("probe_stride", 4)
    c0.set_probe(4)
    pr = c0.run_staged(list(range(min(slots, pool))), bud, ignore_eos=True)
    att = (*c0.get_probe(), *c0.get_probe_device())
    c0.set_probe(0)

    # SURVEY.md §8(d)'s ragged set through the same queue: U[5, 30] s, natural budgets (3.5 tok/s of
    # each utterance's own length), a pool of distinct seeded ragged clips (utterance i = clip i mod pool)
    rpool = min(2 * args.set_pool, n_utt)
    rl = [n for _, n in qd.utterance_set(rpool, args.utt_seed + 1, 5.0, secs)]
    rutts = [(60000 + i, rl[i % rpool]) for i in range(n_utt)]
    with cf.ThreadPoolExecutor(16) as ex:
        rpcm = list(ex.map(lambda i: qasr.synth_pcm(60000 + i, rl[i]), range(rpool)))
    for c in ctxs:
        c.stage_audio(rpcm)
    stats.clear()
    qd.run_queue(stream, rutts[:min(n_utt, 2 * slots * nctx * world)], rank, world, args.tok_rate, dist, dev,
                 key="utt_set_rwarm")
    stats.clear()
    rres = qd.run_queue(stream, rutts, rank, world, args.tok_rate, dist, dev, key="utt_set_rtimed")
    rstats = list(stats)
    for c in ctxs:
        c.close()
    if rank != 0:
        return {}
    toks = res["tokens"]
    assert len(toks) == n_utt and all(len(t) == bud for t in toks.values()), "utterance set: a budget was not met"
    rtoks = rres["tokens"]
    assert len(rtoks) == n_utt and all(len(rtoks[i]) == qd.budget(rutts[i][1], args.tok_rate) for i in range(n_utt)), \
        "ragged utterance set: a budget was not met"
    walls = res["rank_wall_s"]
    hp = m.hp

    # encoder at batch, single context: the probe pass's encoder stage (HIP events around run_encoder)
    ef = min(slots, pool) * encoder_flops(hp, ns)
    enc_s = pr.timings.t_encode_ms / 1e3
    enc = ({"bound": "mfma", "achieved": round(ef / enc_s / 1e12, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ef / enc_s / 1e12 / MFMA_F16_PEAK_TFLOPS, 4), "encoder_ms": round(pr.timings.t_encode_ms, 2),
            "clips": min(slots, pool), "clock": "hip_events, one context alone (untimed pass)"}
           if enc_s > 0 else None)
    # the dominant decode kernel: decode_attn_seq_kernel<1> of layer probe_layer, device clock
    roof = None
    if att[4]:
        avg_s = att[3] / att[4] / 1e3
        bpl = att[2]
        traffic, src = pmc_batch_kernel("void qasr::decode_attn_seq_kernel<1>", min(slots, pool))
        roof = {"kernel": f"decode_attn_seq_kernel<1> (decode batch of {min(slots, pool)}: q/k norm + RoPE + KV write + "
                          f"MFMA scores + ggml fp16-V chain, one workgroup per kv group and sequence), decoder layer "
                          f"{args.probe_layer}",
                "bound": "hbm", "achieved": round(bpl / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(bpl / avg_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
                "bytes_per_launch": round(bpl), "avg_launch_us": round(avg_s * 1e6, 2), "clock": "device",
                "launches": att[4], "pass": "untimed, one context alone"}
    # decode bytes of the timed pass over the contexts' decode time (with the other contexts' refills
    # running beside each one) and of the probe pass alone
    db = set_decode_bytes(hp, timed)
    dsec = sum(st.t_decode_ms for st in timed) / 1e3
    pb = decode_bytes(hp, False, min(slots, pool), P, bud)
    ds1 = pr.timings.t_decode_ms / 1e3
    dh = {"achieved": round(db / dsec / 1e9, 1) if dsec > 0 else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
          "frac": round(db / dsec / 1e9 / HBM_PEAK_GBS, 4) if dsec > 0 else None, "bytes": db,
          "clock": "host, each context's decode chunks (contexts overlapping)",
          "single_context": {"achieved": round(pb / ds1 / 1e9, 1) if ds1 > 0 else None,
                             "frac": round(pb / ds1 / 1e9 / HBM_PEAK_GBS, 4) if ds1 > 0 else None,
                             "bytes": pb, "decode_ms": round(pr.timings.t_decode_ms, 1)}}

    def streams(ss):
        return [{"clips": st.n_clips, "refill_prefills": st.n_prefills, "decode_steps": st.n_steps,
                 "slot_utilisation": round(st.live_steps / max(1, st.slot_steps), 4),
                 "prefill_ms": round(st.t_prefill_ms, 1), "decode_ms": round(st.t_decode_ms, 1),
                 "total_ms": round(st.t_total_ms, 1)} for st in ss]

    def tail(w, ss):   # over ranks (N > 1), else over the rank's contexts
        if len(w) > 1:
            return round((max(w) - min(w)) / max(w), 4) if max(w) > 0 else 0.0
        t = [st.t_total_ms for st in ss]
        return round((max(t) - min(t)) / max(t), 4) if t and max(t) > 0 else 0.0
    rw = rres["rank_wall_s"]
    ragged = {"workload": f"{n_utt} x U[5, {secs:g}] s utterances (a pool of {rpool} distinct seeded ragged clips per "
                          f"GPU, utterance i = clip i mod pool), natural budgets ceil(3.5 tok/s x length), EOS "
                          f"ignored, the same queue and contexts",
              "value": round(rres["audio_s"] / rres["wall_s"], 3), "unit": "audio-sec/wall-sec",
              "audio_s": round(rres["audio_s"], 1), "wall_s": round(rres["wall_s"], 4),
              "decode_tokens_per_s": round(rres["decode_tokens"] / rres["wall_s"], 2),
              "slot_utilisation": round(sum(st.live_steps for st in rstats) / max(1, sum(st.slot_steps for st in rstats)), 4),
              "tail_imbalance": tail(rw, rstats), "per_rank_wall_s": [round(w, 4) for w in rw],
              "rank0_stream": streams(rstats)}
    return {
        "workload": f"configs[3]: {n_utt} x {secs:g} s utterances (16 kHz, a pool of {pool} distinct seeded clips per "
                    f"GPU), one shared longest-first queue feeding {nctx} concurrent continuous-batching context(s) of "
                    f"{slots} slots per GPU (own HIP stream each), "
                    f"greedy budget {bud} tokens (3.5 tok/s), EOS ignored",
        "scaling": "strong", "n_gpus": world, "utterances": n_utt, "audio_s": res["audio_s"],
        "value": round(res["audio_s"] / res["wall_s"], 3), "unit": "audio-sec/wall-sec",
        "wall_s": round(res["wall_s"], 4),
        "decode_tokens_per_s": round(res["decode_tokens"] / res["wall_s"], 2),
        "per_rank_wall_s": [round(w, 4) for w in walls],
        "per_rank_utterances": [int(u) for u in res["rank_utterances"]],
        "tail_imbalance": tail(walls, timed),
        "rank0_stream": streams(timed),
        "roofline": roof,
        "decode_hbm": dh,
        "encoder_roofline": enc,
        "ragged": ragged,
        "collectives": "barrier + max wall time + all_gather of per-rank times and token ids (RCCL); the queue is a "
                       "TCPStore counter (one add per utterance)",
    }


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --gpus counts this node's GPUs: under a multi-node launcher that is LOCAL_WORLD_SIZE, not WORLD_SIZE
    node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.gpus is not None and args.gpus != node:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but this node runs {node} ranks (LOCAL_WORLD_SIZE / WORLD_SIZE)")
    if args.dry_run:
        dry_run(args, world, rank)
        return
    dist = None
    if world > 1:
        # torch ships its own HIP / HSA runtimes (torch/lib): they must initialise before libqasr.so loads,
        # which then binds to torch's libamdhip64.so.7 by soname -- loaded the other way round, two HSA
        # runtimes share the process and the second finds no device (tools/r6/set_run.py RCCL=1)
        assert qasr._lib is None, "libqasr.so loaded before torch's HIP runtime"
        import torch
        import torch.distributed as dist_mod
        torch.cuda.set_device(local)
        dist_mod.init_process_group("nccl")
        dist = dist_mod

    def barrier():
        if dist is not None:
            dist.barrier()

    wtype = 8 if args.q8 else 1
    model_path = args.model or synthetic_model(rank, "full", wtype)
    m = qasr.Model(model_path, local)
    if args.utterances > 0:
        utterance_main(args, m, rank, local, world, dist, model_path)
        if dist is not None:
            dist.destroy_process_group()
        return
    n = int(args.seconds * 16000)
    ntok = int(math.ceil(args.tok_rate * args.seconds))
    T = qasr.mel_frames(n)
    P = qasr.lib().qasr_prompt_len(qasr.encoder_frames(T))
    ctx = qasr.Context(m, max_batch=args.batch, max_ctx=P + ntok + 8)
    clips = [qasr.synth_pcm(1000 + rank * args.batch + i, n) for i in range(args.batch)]
    ctx.stage_audio(clips)
    actx, texts = None, []
    if args.pipeline == "align":   # the ForcedAligner leg: transcript of each clip -> word timestamps
        am = qasr.Model(synthetic_model(rank, "aligner", wtype), local)
        r0 = ctx.run(ntok, ignore_eos=True)
        texts = [m.detokenize(t) for t in r0.tokens]
        need = max(qasr.align_prompt_len(n, len(am.align_tokenize(t)[0])) for t in texts)
        actx = qasr.Context(am, max_batch=min(args.batch, args.align_batch), max_ctx=need + 8)

    def align_all():   # the step's clips, align_batch per aligner pass
        ab = min(args.batch, args.align_batch)
        for k in range(0, len(clips), ab):
            docs, _ = actx.align_json_batch(clips[k:k + ab], texts[k:k + ab])
            assert len(docs) == len(clips[k:k + ab])
    if args.fa_exact_decode is not None:
        ctx.set_option("fa_exact_decode", args.fa_exact_decode)
    fx = ctx.get_option("fa_exact_decode")
    exact = fx != 0
    for _ in range(args.warmup):
        ctx.run(ntok, ignore_eos=True)
        if actx:
            align_all()
    if not args.no_probe:
        ctx.set_option("probe_layer", args.probe_layer)
        # every 8th decode step probed (HIP events + device clock around the
        # group, live in the timed region); the others replay the whole-step
        # graph -- probing every step cost ~3 % of the step time
        ctx.set_option("probe_stride", args.probe_stride)
        ctx.set_probe(2)   # the dominant kernel: layer probe_layer's QKV + attention (+ o-proj) launch
    barrier()
    t0 = time.perf_counter()
    res = None
    tm = {"mel": 0.0, "encode": 0.0, "prefill": 0.0, "decode": 0.0}
    for _ in range(args.steps):
        res = ctx.run(ntok, ignore_eos=True)   # synchronises its stream before returning
        tm["mel"] += res.timings.t_mel_ms
        tm["encode"] += res.timings.t_encode_ms
        tm["prefill"] += res.timings.t_prefill_ms
        tm["decode"] += res.timings.t_decode_ms
        if actx:
            ta = time.perf_counter()
            align_all()
            tm["align"] = tm.get("align", 0.0) + (time.perf_counter() - ta) * 1e3
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    probe = (*ctx.get_probe(), *ctx.get_probe_device()) if not args.no_probe else None
    extra = {}
    if not args.no_probe:   # untimed: one more run per secondary kernel
        for kind in (3, 1):
            ctx.set_probe(kind)
            ctx.run(ntok, ignore_eos=True)
            extra[kind] = (*ctx.get_probe(), *ctx.get_probe_device())
        ctx.set_probe(0)
    assert all(len(x) == ntok for x in res.tokens), "decode budget not met"
    attn_path = ctx.get_option("attn_path")
    # the configs[1] context's HIP stream goes before the utterance set's contexts take theirs: the set
    # contexts + the default stream (+ RCCL's at N > 1) share the box's four hardware queues
    # (GPU_MAX_HW_QUEUES); with it open, three set contexts gave 8590 RTFx against 8768 for two
    ctx.close()
    uset = utterance_set_leg(args, m, rank, local, world, dist) if args.set_utterances > 0 and not actx else None
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    N = world
    audio = N * args.batch * args.seconds * args.steps
    value = audio / dt
    out = {
        "metric": "RTFx (audio-sec/wall-sec) + decode tokens/sec, Qwen3-ASR-0.6B " + ("q8_0" if args.q8 else "f16") +
                  (" + ForcedAligner-0.6B (transcribe-align)" if actx else ""),
        "value": round(value, 3),
        "unit": "audio-sec/wall-sec",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        # published numbers exist only for the f16 clip (ASR, and ASR + align); none for q8_0
        "vs_baseline": None if args.q8 else round(value / (README_ALIGN_RTFX if actx else README_RTFX), 3),
        "dtype": "q8_0 weights, int8 x int8 -> fp32" if args.q8 else "f16",
        "data": f"synthetic (seeded 16 kHz clip; random-init Qwen3-ASR-0.6B-shaped {'q8_0' if args.q8 else 'f16'} GGUF"
                + (", ForcedAligner-0.6B-shaped aligner GGUF)" if actx else ")") if not args.model else
                "synthetic audio; model " + os.path.basename(args.model),
        "config": {"workload": workload(args, ntok, bool(actx)), "clips_per_gpu": args.batch,
                   "clip_seconds": args.seconds, "decode_tokens": ntok, "parallelism": f"dp{N} (utterance sharding)"},
        "decode_tokens_per_s": round(N * args.batch * ntok * args.steps / dt, 2),
        # from the launches the last step actually made (read-only option attn_path)
        "decode_attention": ATTN_LABEL.get(attn_path, "unknown"),
        "stage_ms_per_step_rank0": {k: round(v / args.steps, 3) for k, v in tm.items()},
    }
    if probe and probe[1]:
        # `roofline` = the decode launch with the larger time (both run once per
        # layer per step); the other one and the LM head go to roofline_other
        ents = {2: roofline_entry(2, args.batch, *probe, args.probe_layer, exact, args.q8)}
        ents.update({k: roofline_entry(k, args.batch, *v, args.probe_layer, exact, args.q8) for k, v in extra.items()
                     if v[1]})
        top = max((k for k in ents if k != 1), key=lambda k: ents[k]["avg_launch_us"])
        out["roofline"] = ents.pop(top)
        out["roofline_other"] = list(ents.values())
    # the north-star fractions of the two stages: encoder
    # FLOPs against the dense fp16 MFMA peak, decode bytes against HBM
    enc_s = tm["encode"] / args.steps / 1e3
    if enc_s > 0:
        ef = args.batch * encoder_flops(m.hp, n)
        out["encoder_roofline"] = {"bound": "mfma", "achieved": round(ef / enc_s / 1e12, 1), "peak": MFMA_F16_PEAK_TFLOPS,
                                   "unit": "TFLOP/s", "frac": round(ef / enc_s / 1e12 / MFMA_F16_PEAK_TFLOPS, 4),
                                   "flops_per_step": ef, "profiled": profiled_mfma()}
    dec_s = tm["decode"] / args.steps / 1e3
    if dec_s > 0:
        db = decode_bytes(m.hp, args.q8, args.batch, P, ntok)
        out["decode_hbm"] = {"achieved": round(db / dec_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(db / dec_s / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_step": db}
    if uset:
        out["utterance_set"] = uset
    if N == 1 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(model_path, args.cpu_sample_seconds, args.tok_rate, args.cpu_threads,
                                           args.seconds, ntok)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
