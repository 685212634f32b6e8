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


def test_utterance_set_and_batches():
    from qasr_dist import batches_of, budget, utterance_set
    u = utterance_set(1000, seed=0)
    assert len(u) == 1000 and len({s for s, _ in u}) == 1000
    secs = [n / 16000 for _, n in u]
    assert 5.0 <= min(secs) and max(secs) <= 30.0 and all(n % 160 == 0 for _, n in u)
    assert utterance_set(1000, seed=0) == u and utterance_set(1000, seed=1) != u
    assert budget(30 * 16000, 3.5) == 105 and budget(92 * 16000, 3.5) == 322
    lens = [n for _, n in u]
    b = batches_of(list(range(100)), lens, 64)
    assert [len(x) for x in b] == [64, 36]
    assert all(lens[x[i]] >= lens[x[i + 1]] for x in b for i in range(len(x) - 1))


def _driver_worker(rank, world, port, q):
    """the full sharded driver loop with a stub transcriber (token k of
    utterance i = i * 1000 + k): sharding, per-utterance budgets, timing,
    gather to rank 0"""
    import torch.distributed as dist
    from qasr_dist import run_shard, utterance_set
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    utts = utterance_set(37, seed=3)
    calls = []

    def transcribe(idx, max_tokens):
        calls.append((list(idx), max_tokens))
        return [[i * 1000 + k for k in range(max_tokens)] for i in idx]

    res = run_shard(transcribe, utts, rank, world, batch=8, tok_rate=3.5, dist=dist)
    q.put((rank, res["tokens"], res["wall_s"], sorted(res["local"]), calls))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_driver(world):
    import math
    import torch.multiprocessing as mp
    from qasr_dist import utterance_set
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_driver_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    utts = utterance_set(37, seed=3)
    want = {i: [i * 1000 + k for k in range(math.ceil(3.5 * n / 16000))] for i, (_, n) in enumerate(utts)}
    assert res[0][1] == want and all(r[1] is None for r in res[1:])
    assert len({r[2] for r in res}) == 1   # one max-over-ranks wall time
    shards = [r[3] for r in res]
    assert sorted(i for s in shards for i in s) == list(range(37))
    for _, _, _, mine, calls in res:   # batches of <= 8, each decoded to its longest clip's budget
        assert all(len(idx) <= 8 and mt == max(math.ceil(3.5 * utts[i][1] / 16000) for i in idx) for idx, mt in calls)
        assert sorted(i for idx, _ in calls for i in idx) == mine


def _queue_worker(rank, world, port, q):
    import time as _t
    import torch.distributed as dist
    from qasr_dist import budget, run_queue
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    utts = [(1000 + i, (5 + 3 * i) * 16000) for i in range(11)]

    def stream(next_clip):   # a stand-in for Context.run_stream_staged: rank 1 is 3x slower per clip
        out = {}
        while True:
            item = next_clip()
            if item is None:
                return out
            i, b = item
            _t.sleep(0.01 * (1 + 2 * rank))
            out[i] = [i] * b
    res = run_queue(stream, utts, rank, world, 3.5, dist, key="qtest")
    # every rank's own stream time and utterance count, gathered (the bench's tail imbalance)
    assert len(res["rank_wall_s"]) == world and res["rank_wall_s"][rank] <= res["wall_s"]
    assert res["rank_utterances"][rank] == len(res["local"]) and sum(res["rank_utterances"]) == len(utts)
    q.put((rank, sorted(res["local"]), res["tokens"]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_dynamic_queue():
    """run_queue: the shared TCPStore counter hands every utterance to exactly
    one rank, the faster rank takes more, rank 0 gathers all of them"""
    import torch.multiprocessing as mp
    from qasr_dist import budget
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_queue_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, l0, m0), (_, l1, m1) = res
    assert sorted(l0 + l1) == list(range(11)) and not set(l0) & set(l1)
    assert len(l0) > len(l1)
    assert m1 is None
    assert m0 == {i: [i] * budget((5 + 3 * i) * 16000, 3.5) for i in range(11)}


def test_queue_order_and_local_counter():
    from qasr_dist import make_next, queue_order
    lens = [16000 * s for s in (5, 30, 12, 30, 7)]
    assert queue_order(lens) == [1, 3, 2, 4, 0]
    nxt = make_next(queue_order(lens), lens, 3.5)
    got = [nxt() for _ in range(6)]
    assert [g[0] for g in got[:5]] == [1, 3, 2, 4, 0] and got[5] is None
    assert got[0][1] == 105


def test_bench_launcher_spawns_ranks():
    """`python bench.py --gpus 2` without torchrun spawns two ranks itself
    (bench.launch_ranks) and prints exactly one JSON line, rank 0's, with
    n_gpus = 2 (dry run: gloo rendezvous, no GPU)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["parallelism"] == "dp2"


def test_bench_launcher_propagates_failure():
    """a rank that exits non-zero makes the launcher exit non-zero: rank 1
    dies before the rendezvous (QASR_BENCH_FAIL_RANK), rank 0 is terminated"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=dict(env, QASR_BENCH_FAIL_RANK="1"))
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def test_bench_batch_group_traffic(tmp_path, monkeypatch):
    """bench.pmc_group_traffic: the batch launch groups' HBM bytes per
    layer-step from a batch PMC summary -- attention + the once-per-layer
    plain-epilogue skinny GEMM (QKV) to group 2, the SwiGLU and o/down
    instances to group 3, rmsnorm left out, other batch sizes ignored."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    d = tmp_path / "profiles" / "r9" / "batch" / "f16"
    d.mkdir(parents=True)
    k = lambda n, c, r, w: {"name": n, "calls": c, "avg_us": 1.0, "total_ms": 1.0, "hbm_read_bytes": r, "hbm_write_bytes": w}
    (d / "summary.json").write_text(json.dumps({"kernels": [
        k("void qasr::decode_attn_seq_kernel<1>(qasr::DecodeAttnArgs)", 10, 100, 1),
        k("void qasr::gemm_skinny_kernel<4, 1, 8, 0, 4, 2>(qasr::GemmArgs)", 10, 20, 2),
        k("void qasr::gemm_skinny_kernel<2, 2, 4, 2, 4, 2>(qasr::GemmArgs)", 10, 30, 3),
        k("void qasr::gemm_skinny_kernel<1, 1, 8, 0, 4, 2>(qasr::GemmArgs)", 20, 10, 1),
        k("void qasr::rmsnorm_kernel<1024>(float const*)", 21, 1000, 1000)]}))
    (d / "bench.json").write_text(json.dumps({"config": {"clips_per_gpu": 64}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_group_traffic(2, 64, False) == (123, "profiles/r9/batch/f16/summary.json")
    assert bench.pmc_group_traffic(3, 64, False) == (33 + 22, "profiles/r9/batch/f16/summary.json")
    assert bench.pmc_group_traffic(2, 32, False) == (None, None)
    assert bench.pmc_group_traffic(2, 64, True) == (None, None)


def test_bench_gpus_counts_this_node_under_a_multinode_launch():
    """--gpus is this node's GPU count -- under a launcher that is
    LOCAL_WORLD_SIZE, not WORLD_SIZE.  Four ranks as two 'nodes' of two
    (WORLD_SIZE = 4, LOCAL_WORLD_SIZE = 2) each run `bench.py --gpus 2
    --dry-run`: all four join the gloo group and rank 0 prints n_gpus = 4;
    --gpus 4 on the same layout is refused before any work."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import bench_port
    port = bench_port.free_port()
    base = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "LOCAL_WORLD_SIZE")}

    def launch(gpus):
        ps = []
        for r in range(4):
            env = dict(base, WORLD_SIZE="4", RANK=str(r), LOCAL_RANK=str(r % 2), LOCAL_WORLD_SIZE="2",
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            ps.append(subprocess.Popen([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--dry-run"],
                                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        return [(p.wait(timeout=300), *p.communicate()) for p in ps]
    outs = launch(2)
    assert all(rc == 0 for rc, _, _ in outs), [e[-800:] for _, _, e in outs]
    lines = [ln for _, o, _ in outs for ln in o.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 4, lines
    bad = launch(4)
    assert all(rc != 0 and "LOCAL_WORLD_SIZE" in e for rc, _, e in bad), [(rc, e[-300:]) for rc, _, e in bad]


def test_set_contexts_policy():
    """bench.set_contexts (round 6, profiles/r6/set_contexts.txt and
    set_contexts_r6b.txt): contexts per GPU by the rank's share of the
    utterance set -- 1 x 125 at N = 8, 2 x 125 at N = 4, 4 x 125 at N = 2,
    4 x 128 at N = 1"""
    import bench
    assert [bench.set_contexts(-(-1000 // n)) for n in (1, 2, 4, 8)] == [4, 4, 2, 1]
    assert bench.set_contexts(128) == 1 and bench.set_contexts(129) == 2 and bench.set_contexts(256) == 2
    assert bench.set_contexts(257) == 4 and bench.set_contexts(10000) == 4


def test_bench_raises_hw_queues():
    """bench.py asks the HIP runtime for 8 hardware queues a process (set before
    any GPU call; the utterance set's context streams share HIP's default 4)"""
    import os
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-c", "import os, bench; print(os.environ['GPU_MAX_HW_QUEUES'])"],
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         env={k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"},
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "8", (out.stdout, out.stderr[-500:])
