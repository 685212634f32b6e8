"""Continuous batching (qasr_run_stream): slots refilled from a queue.

The reference transcribes one utterance at a time (src/qwen3_asr.cpp:270-296),
so a clip's tokens must not depend on which clips share its batch or when its
slot was refilled: every clip of a stream run equals a one-clip qasr_run of
the same clip and budget.  Ragged per-clip budgets stand in for natural EOS
(random-init weights rarely emit it) and make the refill schedule
deterministic; slot-steps must drop against static batches run to their
longest member.
"""
import numpy as np
import pytest

import qasr

SR = 16000
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny_model(gpu, tiny_gguf):
    m = qasr.Model(tiny_gguf)
    yield m
    m.close()


def _single(m, pcm, budget, ignore_eos):
    c = qasr.Context(m, max_batch=1, max_ctx=640)
    try:
        return c.transcribe([pcm], max_tokens=budget, ignore_eos=ignore_eos).tokens[0]
    finally:
        c.close()


def _queue(items):
    it = iter(items)
    return lambda: next(it, None)


@pytest.mark.parametrize("slots", [3, 1])
def test_stream_ragged_budgets_equal_single(tiny_model, slots):
    lens = [SR, 2 * SR + 333, 4 * SR, SR // 2, 3 * SR, 5 * SR + 7, SR + 999]
    budgets = [3, 9, 5, 16, 1, 7, 12]
    clips = [qasr.synth_pcm(7100 + i, n) for i, n in enumerate(lens)]
    c = qasr.Context(tiny_model, max_batch=slots, max_ctx=640)
    try:
        out, st = c.run_stream(_queue([(10 + i, p, b) for i, (p, b) in enumerate(zip(clips, budgets))]), max_tokens=32,
                               ignore_eos=True)
    finally:
        c.close()
    assert sorted(out) == [10 + i for i in range(len(clips))]
    for i, (p, b) in enumerate(zip(clips, budgets)):
        assert out[10 + i] == _single(tiny_model, p, b, True), i
        assert len(out[10 + i]) == b
    assert st.n_clips == len(clips) and st.n_errors == 0
    # every live slot-step produced one token after the prefill's
    assert st.live_steps == sum(budgets) - len(clips)
    # static batches of `slots` clips in queue order, each run to its longest budget
    static = sum(slots * (max(budgets[k:k + slots]) - 1) for k in range(0, len(budgets), slots))
    assert st.slot_steps < static or slots == 1


def test_stream_refill_groups_equal_single(tiny_model):
    """option refill_group: at most g clips a refill, decode
    steps between the groups -- a different schedule, the same tokens per clip"""
    lens = [SR, 2 * SR + 333, 4 * SR, SR // 2, 3 * SR, 5 * SR + 7, SR + 999, 2 * SR]
    budgets = [3, 9, 5, 16, 1, 7, 12, 10]
    clips = [qasr.synth_pcm(7150 + i, n) for i, n in enumerate(lens)]
    c = qasr.Context(tiny_model, max_batch=5, max_ctx=640)
    try:
        c.set_option("refill_group", 2)
        out, st = c.run_stream(_queue([(30 + i, p, b) for i, (p, b) in enumerate(zip(clips, budgets))]), max_tokens=32,
                               ignore_eos=True)
    finally:
        c.close()
    for i, (p, b) in enumerate(zip(clips, budgets)):
        assert out[30 + i] == _single(tiny_model, p, b, True), i
    assert st.n_clips == len(clips) and st.n_prefills >= 4   # groups of at most 2


def test_stream_live_prefix_batches_equal_single(tiny_model):
    """option live_prefix: decode chunks run over the slots up to the last live
    one (16-row granules) -- with refill groups of 5 into 40 slots the chunks
    switch between 16-, 32- and 40-row batches; every clip's tokens equal its
    one-clip run"""
    n = 23
    lens = [SR // 2 + 2311 * i for i in range(n)]
    budgets = [2 + (7 * i) % 13 for i in range(n)]
    clips = [qasr.synth_pcm(7170 + i, m) for i, m in enumerate(lens)]
    c = qasr.Context(tiny_model, max_batch=40, max_ctx=640)
    try:
        c.set_option("refill_group", 5)
        c.set_option("live_prefix", 1)
        out, st = c.run_stream(_queue([(50 + i, p, b) for i, (p, b) in enumerate(zip(clips, budgets))]), max_tokens=32,
                               ignore_eos=True)
    finally:
        c.close()
    for i, (p, b) in enumerate(zip(clips, budgets)):
        assert out[50 + i] == _single(tiny_model, p, b, True), i
    assert st.n_clips == n and st.n_prefills >= 5


def test_stream_natural_eos_and_per_clip_errors(tiny_model):
    good = [qasr.synth_pcm(7200 + i, n) for i, n in enumerate([SR, 3 * SR, 2 * SR])]
    items = [(0, good[0], 8), (1, qasr.synth_pcm(7300, 100), 8), (2, good[1], 8), (3, qasr.synth_pcm(7301, SR), 10000),
             (4, good[2], 6)]
    c = qasr.Context(tiny_model, max_batch=2, max_ctx=640)
    try:
        out, st = c.run_stream(_queue(items), max_tokens=8, ignore_eos=False)
    finally:
        c.close()
    assert isinstance(out[1], qasr.QasrError) and "audio_pad" in str(out[1])
    assert isinstance(out[3], qasr.QasrError) and "Context length" in str(out[3])
    for cid, pcm, b in (items[0], items[2], items[4]):
        assert out[cid] == _single(tiny_model, pcm, b, False), cid
        assert 151645 not in out[cid]
    assert st.n_clips == 3 and st.n_errors == 2


def test_stream_token_callback_gets_clip_ids(tiny_model):
    clips = [qasr.synth_pcm(7400 + i, SR + 500 * i) for i in range(3)]
    seen = {}
    c = qasr.Context(tiny_model, max_batch=2, max_ctx=640)
    try:
        c.set_token_callback(lambda cid, n, tok: seen.setdefault(cid, []).append((n, tok)))
        out, _ = c.run_stream(_queue([(40 + i, p, 4 + i) for i, p in enumerate(clips)]), max_tokens=16, ignore_eos=True)
        c.set_token_callback(None)
    finally:
        c.close()
    for cid, toks in out.items():
        assert [n for n, _ in seen[cid]] == list(range(1, len(toks) + 1))
        assert [t for _, t in seen[cid]] == toks


def test_stream_fetch_exception_is_raised(tiny_model):
    """a Python exception inside next_clip() (ctypes would swallow it and the
    engine take 0 as a clip id) closes the queue and is re-raised after the
    run; the clips fetched before it are still transcribed"""
    clips = [qasr.synth_pcm(7400 + i, SR) for i in range(3)]
    calls = []

    def next_clip():
        calls.append(1)
        if len(calls) == 3:
            raise RuntimeError("queue store failed")
        return (len(calls), clips[len(calls) - 1], 4) if len(calls) < 3 else None

    c = qasr.Context(tiny_model, max_batch=2, max_ctx=640)
    try:
        with pytest.raises(RuntimeError, match="queue store failed"):
            c.run_stream(next_clip, max_tokens=4, ignore_eos=True)
        c.stage_audio(clips)
        with pytest.raises(ValueError, match="bad index"):
            c.run_stream_staged(lambda: (_ for _ in ()).throw(ValueError("bad index")), max_tokens=4, ignore_eos=True)
        # the context stays usable
        out, st = c.run_stream(_queue([(5, clips[0], 4)]), max_tokens=4, ignore_eos=True)
        assert out[5] == _single(tiny_model, clips[0], 4, True)
    finally:
        c.close()


def test_stream_staged_ids_outside_pool(tiny_model):
    """a staged id outside the pool fails that clip (out of range)
    unless option staged_wrap asks for id % pool reuse (bench.py's utterance
    sets over a 128-clip pool); the other clips are transcribed either way"""
    clips = [qasr.synth_pcm(7500 + i, SR + 300 * i) for i in range(2)]
    c = qasr.Context(tiny_model, max_batch=2, max_ctx=640)
    try:
        c.stage_audio(clips)
        out, st = c.run_stream_staged(_queue([0, 5, 1]), max_tokens=4, ignore_eos=True)
        assert isinstance(out[5], qasr.QasrError) and "out of range" in str(out[5])
        assert st.n_errors == 1 and out[0] == _single(tiny_model, clips[0], 4, True)
        c.set_option("staged_wrap", 1)
        out, st = c.run_stream_staged(_queue([0, 5, 1]), max_tokens=4, ignore_eos=True)
        assert st.n_errors == 0 and out[5] == out[1] == _single(tiny_model, clips[1], 4, True)
    finally:
        c.close()


def test_concurrent_streams_equal_single(tiny_model):
    """bench.py's utterance_set runs several continuous-batching contexts of one
    model at once, each on its own HIP stream and host thread, fed by one
    locked queue: every clip's tokens equal its one-clip run whichever context
    took it, and every clip is delivered exactly once."""
    import concurrent.futures as cf
    import threading
    lens = [SR + 160 * i for i in range(10)]
    budgets = [4 + (i % 5) for i in range(10)]
    clips = [qasr.synth_pcm(7300 + i, n) for i, n in enumerate(lens)]
    items = iter([(20 + i, p, b) for i, (p, b) in enumerate(zip(clips, budgets))])
    lock = threading.Lock()

    def take():
        with lock:
            return next(items, None)
    ctxs = [qasr.Context(tiny_model, max_batch=3, max_ctx=640) for _ in range(2)]
    try:
        with cf.ThreadPoolExecutor(2) as ex:
            res = list(ex.map(lambda c: c.run_stream(take, max_tokens=16, ignore_eos=True), ctxs))
    finally:
        for c in ctxs:
            c.close()
    out = {}
    for o, st in res:
        assert not set(o) & set(out)
        out.update(o)
    assert sorted(out) == [20 + i for i in range(len(clips))]
    for i, (p, b) in enumerate(zip(clips, budgets)):
        assert out[20 + i] == _single(tiny_model, p, b, True), i


def test_env_eager_and_trace_paths_equal_default(tiny_model, tmp_path, monkeypatch):
    """the environment switches outside fuse_options().
    QASR_NO_GRAPH=1 (decode steps launched eagerly, for profilers) and
    QASR_DEV_TRACE (per-block timestamps of one layer's kernels) change how the
    step is launched, never what it computes: tokens of a batch-1 and a
    batch-3 run equal the default context's, and the trace file is written."""
    clips = [qasr.synth_pcm(7600 + i, SR + 700 * i) for i in range(3)]

    def run():
        c = qasr.Context(tiny_model, max_batch=3, max_ctx=640)
        try:
            return (c.transcribe(clips[:1], max_tokens=10, ignore_eos=True).tokens,
                    c.transcribe(clips, max_tokens=10, ignore_eos=True).tokens)
        finally:
            c.close()
    base = run()
    monkeypatch.setenv("QASR_NO_GRAPH", "1")
    assert run() == base
    monkeypatch.delenv("QASR_NO_GRAPH")
    tr = tmp_path / "trace.bin"
    monkeypatch.setenv("QASR_DEV_TRACE", str(tr))
    monkeypatch.setenv("QASR_DEV_TRACE_LAYER", "0")
    assert run() == base
    assert tr.exists() and tr.stat().st_size > 0
