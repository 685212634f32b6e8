"""qasr_dist -- utterance-level data parallelism.

One process per GPU; utterances are independent, so each rank transcribes its
own shard with no collective on the data path.  torch.distributed (RCCL over
xGMI on the GPU box, gloo in CPU tests) is used only to
  - synchronise the timed region (barrier) and take the max wall time,
  - gather the per-utterance token-id arrays to rank 0 at the end
    (allgather of lengths + one padded int32 gather: KBs per utterance).
"""
from __future__ import annotations

from typing import List, Sequence

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
