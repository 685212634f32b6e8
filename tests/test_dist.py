"""CPU: the multi-GPU (utterance-sharded) path with torch.distributed gloo,
world_size 2 -- sharding, max-over-ranks timing, token gather to rank 0."""
import os
import socket

import pytest

from qasr_dist import gather_tokens, max_over_ranks, shard_longest_first


def test_shard_longest_first_balanced():
    lens = [30, 5, 92, 30, 12, 7, 30, 61]
    for world in (1, 2, 3, 8):
        sh = shard_longest_first(lens, world)
        flat = sorted(i for s in sh for i in s)
        assert flat == list(range(len(lens)))
        loads = [sum(lens[i] for i in s) for s in sh]
        assert max(loads) - min(loads) <= max(lens)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens = [30 * 16000, 5 * 16000, 92 * 16000, 7 * 16000, 11 * 16000]
    mine = shard_longest_first(lens, world)[rank]
    local = {i: [i * 10 + k for k in range(i + 1)] for i in mine}
    t = max_over_ranks(1.0 + rank, dist)
    merged = gather_tokens(local, dist)
    q.put((rank, t, merged))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_and_max():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, t0, m0), (r1, t1, m1) = res
    assert t0 == t1 == 2.0
    assert m1 is None
    assert m0 == {i: [i * 10 + k for k in range(i + 1)] for i in range(5)}
