"""qasr_dist -- utterance-level data parallelism.

One process per GPU; utterances are independent, so each rank transcribes
utterances with no collective on the data path (configs[3]: a 1000-utterance
f16 batch sharded over the node's GPUs; configs[4]: the same with the
ForcedAligner leg on every utterance).  The reference's only batch mode is a
shell loop over files (docs/usage.md:240-252); this is its sharded
counterpart.  torch.distributed (RCCL over
xGMI on the GPU box, gloo in CPU tests) is used only to
  - synchronise the timed region (barrier) and take the max wall time,
  - gather the per-utterance token-id arrays to rank 0 at the end
    (allgather of lengths + one padded int32 gather: KBs per utterance).
Two drivers: run_queue (default) -- a dynamic work queue, one shared counter
in the process group's TCPStore (store.add per utterance, longest first), each
rank's continuous-batching stream pulling the next utterance whenever a slot
frees; run_shard -- the static longest-first split in fixed batches.
"""
from __future__ import annotations

import math
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np


def shard_longest_first(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment of utterance indices to
    ranks (balances total audio per GPU; tail imbalance <= one utterance)."""
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    load = [0] * world
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += int(lengths[i])
    for s in shards:
        s.sort()
    return shards


def max_over_ranks(value: float, dist, device=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_floats(value: float, dist, device=None) -> List[float]:
    """every rank's value (rank order), on every rank"""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [float(value)]
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def gather_tokens(local: dict, dist, device=None):
    """local: {utterance_index: [token ids]} on every rank.  Returns the merged
    dict on rank 0 (None elsewhere).  Two collectives: an all_gather of the
    per-rank payload sizes, then one all_gather of the padded int32 payloads."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(local)
    import torch
    world = dist.get_world_size()
    flat: List[int] = []
    for idx, toks in sorted(local.items()):
        flat += [int(idx), len(toks)] + [int(t) for t in toks]
    n = torch.tensor([len(flat)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    cap = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(max(cap, 1), dtype=torch.int32, device=device)
    if flat:
        buf[:len(flat)] = torch.tensor(flat, dtype=torch.int32, device=device)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    if dist.get_rank() != 0:
        return None
    out = {}
    for r in range(world):
        a = bufs[r][:int(sizes[r].item())].cpu().numpy().astype(np.int64)
        p = 0
        while p < len(a):
            idx, ln = int(a[p]), int(a[p + 1])
            out[idx] = a[p + 2:p + 2 + ln].tolist()
            p += 2 + ln
    return out


def utterance_set(n: int, seed: int = 0, lo: float = 5.0, hi: float = 30.0, sr: int = 16000) -> List[Tuple[int, int]]:
    """n seeded utterances: (pcm seed, samples), lengths
    U[lo, hi] seconds (lo == hi: fixed length), whole 10 ms hops."""
    rng = np.random.default_rng(seed)
    secs = rng.uniform(lo, hi, n) if hi > lo else np.full(n, lo)
    return [(1000 + i, int(round(float(s) * 100)) * (sr // 100)) for i, s in enumerate(secs)]


def budget(samples: int, tok_rate: float, sr: int = 16000) -> int:
    """fixed greedy decode budget: ceil(tok_rate x seconds)"""
    return max(1, int(math.ceil(tok_rate * samples / sr)))


def batches_of(shard: Sequence[int], lengths: Sequence[int], batch: int) -> List[List[int]]:
    """a rank's utterances longest first, cut into batches of similar length
    (each batch decodes to its longest clip's budget; sorted, that overshoot
    stays small)"""
    order = sorted(shard, key=lambda i: (-int(lengths[i]), i))
    return [order[k:k + batch] for k in range(0, len(order), batch)]


def run_shard(transcribe: Callable[[List[int], int], List[List[int]]], utts: Sequence[Tuple[int, int]], rank: int,
              world: int, batch: int, tok_rate: float, dist=None, device=None,
              after_batch: Optional[Callable[[List[int], List[List[int]]], None]] = None) -> Dict:
    """The sharded data-parallel driver.  transcribe(indices, max_tokens) ->
    token lists for those utterances (already staged by the caller, e.g. in
    HBM); each utterance keeps its own budget's worth of tokens.  Barrier ->
    timed pass over this rank's batches -> barrier; the wall time is the max
    over ranks; the token ids are gathered to rank 0 (the only collectives).
    Returns {"tokens" (rank 0: all utterances), "wall_s", "audio_s",
    "decode_tokens", "local"}."""
    lengths = [n for _, n in utts]
    shard = shard_longest_first(lengths, world)[rank]
    plan = batches_of(shard, lengths, batch)
    if dist is not None and dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    local: Dict[int, List[int]] = {}
    for idx in plan:
        toks = transcribe(idx, max(budget(lengths[i], tok_rate) for i in idx))
        for i, t in zip(idx, toks):
            local[i] = list(t[:budget(lengths[i], tok_rate)])
        if after_batch is not None:
            after_batch(idx, [local[i] for i in idx])
    if dist is not None and dist.is_initialized():
        dist.barrier()
    wall = max_over_ranks(time.perf_counter() - t0, dist, device)
    merged = gather_tokens(local, dist, device)
    return {"tokens": merged, "wall_s": wall, "audio_s": sum(lengths) / 16000.0,
            "decode_tokens": sum(budget(n, tok_rate) for n in lengths), "local": local, "batches": len(plan)}


def queue_order(lengths: Sequence[int]) -> List[int]:
    """the shared queue's order: longest first (ties by index)"""
    return sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))


def make_next(order: Sequence[int], lengths: Sequence[int], tok_rate: float, store=None, key: str = "q"):
    """next_clip() for a rank's stream: the k-th utterance of `order`, k from
    store.add(key, 1) (shared by every rank: a dynamic queue) or a local
    counter (one rank); (index, budget) or None when the queue is drained"""
    local = [0]

    def next_clip():
        if store is not None:
            k = int(store.add(key, 1)) - 1
        else:
            k = local[0]
            local[0] += 1
        if k >= len(order):
            return None
        i = order[k]
        return i, budget(lengths[i], tok_rate)
    return next_clip


def default_store(dist):
    """the TCPStore of the default process group (None: one process)"""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return None
    from torch.distributed import distributed_c10d
    return distributed_c10d._get_default_store()


def run_queue(stream: Callable[[Callable], Dict[int, List[int]]], utts: Sequence[Tuple[int, int]], rank: int, world: int,
              tok_rate: float, dist=None, device=None, key: str = "q",
              after: Optional[Callable[[List[int], List[List[int]]], None]] = None) -> Dict:
    """The dynamic-queue driver.  stream(next_clip) -> {index: tokens} runs
    this rank's continuous-batching stream until next_clip() is None
    (qasr.Context.run_stream_staged).  key: a fresh store key per pass.
    Barrier -> timed stream (+ after(indices, tokens), e.g. the aligner) ->
    barrier; wall = max over ranks; tokens gathered to rank 0."""
    lengths = [n for _, n in utts]
    store = default_store(dist)
    next_clip = make_next(queue_order(lengths), lengths, tok_rate, store, key)
    if dist is not None and dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    local = dict(stream(next_clip))
    if after is not None and local:
        idx = sorted(local)
        after(idx, [local[i] for i in idx])
    own = time.perf_counter() - t0   # this rank's stream (+ after) done: its own wall time, before the barrier
    if dist is not None and dist.is_initialized():
        dist.barrier()
    wall = max_over_ranks(time.perf_counter() - t0, dist, device)
    rank_walls = gather_floats(own, dist, device)
    merged = gather_tokens(local, dist, device)
    return {"tokens": merged, "wall_s": wall, "audio_s": sum(lengths) / 16000.0,
            "decode_tokens": sum(budget(n, tok_rate) for n in lengths), "local": local, "batches": None,
            "rank_wall_s": rank_walls, "rank_utterances": gather_floats(len(local), dist, device)}
