"""GPU: the boundary's host-facing features beyond the hot path's numerics --
per-token callback, --profile sections, staged pools run in subsets, the CLI's
sharded --devices / --file-list mode, and the sharded bench driver."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import qasr

pytestmark = pytest.mark.gpu
SR = 16000
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "qwen3-asr.cpp_amd", "qwen3-asr-cli")


@pytest.fixture(scope="module")
def tiny(gpu, tiny_gguf):
    m = qasr.Model(tiny_gguf)
    c = qasr.Context(m, max_batch=4, max_ctx=256)
    yield m, c
    c.close()
    m.close()


def test_token_callback_is_per_token(tiny):
    """src/qwen3_asr.cpp:255-291: called after every token, the prefill's
    first, with the running count; the delivered ids are the result's."""
    m, c = tiny
    clips = [qasr.synth_pcm(31000 + i, (2 + i) * SR) for i in range(2)]
    seen = {0: [], 1: []}
    c.set_token_callback(lambda seq, n, tok: seen[seq].append((n, tok)))
    try:
        r = c.transcribe(clips, max_tokens=12, ignore_eos=True)
    finally:
        c.set_token_callback(None)
    for b in range(2):
        assert [n for n, _ in seen[b]] == list(range(1, 13))
        assert [t for _, t in seen[b]] == r.tokens[b]
    assert c.transcribe(clips, max_tokens=12, ignore_eos=True).tokens == r.tokens   # no callback: same ids


def test_token_callback_stops_at_eos(tiny):
    m, c = tiny
    pcm = qasr.synth_pcm(31500, 2 * SR)
    seen = []
    c.set_token_callback(lambda seq, n, tok: seen.append(tok))
    try:
        r = c.transcribe([pcm], max_tokens=40)
    finally:
        c.set_token_callback(None)
    eos = m.hp.eos_id
    if seen and seen[-1] == eos:
        assert seen[:-1] == r.tokens[0]   # trailing EOS popped from the result (src/qwen3_asr.cpp:298-300)
    else:
        assert seen == r.tokens[0] and len(seen) == 40


def test_profile_sections(tiny):
    m, c = tiny
    c.set_profile(True)
    try:
        c.transcribe([qasr.synth_pcm(31600, 3 * SR)], max_tokens=9, ignore_eos=True)
        rep = c.profile_report()
    finally:
        c.set_profile(False)
    assert "TIMING PROFILE REPORT" in rep
    rows = {ln.split()[0]: ln.split()[1:] for ln in rep.splitlines() if ln[:1].isalpha() and not ln.startswith("Section")}
    for k in ("mel_spectrogram", "audio_encoding.total", "audio_encoding.conv_chunk", "audio_encoding.transformer",
              "decode.initial_forward", "decode.token", "transcribe.total"):
        assert k in rows, (k, rep)
    assert int(rows["decode.token"][1]) == 8
    assert float(rows["transcribe.total"][0]) > 0


def test_staged_pool_subsets(tiny):
    """qasr_run_staged: a pool larger than max_batch, run in subsets, gives
    the same ids as each clip alone"""
    m, c = tiny
    clips = [qasr.synth_pcm(32000 + i, int((1.5 + 0.7 * i) * SR)) for i in range(6)]
    alone = [c.transcribe([x], max_tokens=6, ignore_eos=True).tokens[0] for x in clips]
    c.stage_audio(clips)
    with pytest.raises(qasr.QasrError):
        c.run(6, ignore_eos=True)   # 6 staged > max_batch 4
    got = {}
    for sub in ([0, 2], [5, 1, 3, 4]):
        r = c.run_staged(sub, 6, ignore_eos=True)
        got.update(zip(sub, r.tokens))
    assert [got[i] for i in range(6)] == alone


def test_cli_sharded_file_list(tiny, tmp_path, tiny_gguf):
    """qwen3-asr-cli --devices / --file-list / --batch: outputs in input
    order, identical to one file at a time (a 40 s file included: the
    sharded stream sizes its context to the longest file up to 120 s; the
    130 s file goes to the long-file queue, its own context -- ADVICE r4);
    --profile prints the report"""
    paths = []
    for i, secs in enumerate((1.2, 2.2, 40.0, 130.0, 3.2)):
        p = str(tmp_path / f"c{i}.wav")
        qasr.write_wav(p, qasr.synth_pcm(33000 + i, int(secs * SR)))
        paths.append(p)
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(paths) + "\n")
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(CLI))
    one = []
    for p in paths:
        r = subprocess.run([CLI, "-m", tiny_gguf, "-f", p, "--max-tokens", "8", "--no-timing"], capture_output=True,
                           text=True, env=env, timeout=120)
        assert r.returncode == 0, r.stderr
        one.append(r.stdout)
    r = subprocess.run([CLI, "-m", tiny_gguf, "--devices", "0", "--file-list", str(lst), "--batch", "2",
                        "--max-tokens", "8"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout == "".join(one)
    assert "Sharded timing" in r.stderr
    r = subprocess.run([CLI, "-m", tiny_gguf, "-f", paths[0], "--max-tokens", "8", "--profile"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0 and "TIMING PROFILE REPORT" in r.stderr and "decode.token" in r.stderr


@pytest.mark.parametrize("queue,pipeline,n", [("dynamic", "asr", 24), ("static", "asr", 24), ("dynamic", "align", 48)])
def test_bench_utterance_driver(gpu, queue, pipeline, n, tmp_path):
    """bench.py --utterances (configs[3] driver; configs[4] with --pipeline
    align) at a small size, full-size synthetic models: every utterance
    transcribed to its budget (bench.py asserts it), with align every
    transcript aligned; one JSON line, strong scaling.  dynamic: the shared
    queue feeding the continuous-batching stream.  align: rank 0's shortest
    utterance's document from the driver (--dump-align) against the oracle's
    aligner on the same clip and transcript: the same words, and each
    timestamp the oracle's class x 80 ms (LIS-repaired) wherever the oracle's
    own top-1/top-2 margin is clear of its noise floor (tests/test_gpu_aligner.py)."""
    dump = str(tmp_path / "align.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--utterances", str(n), "--utt-min", "2",
                        "--utt-max", "6", "--batch", "8", "--steps", "1", "--warmup", "1", "--queue", queue,
                        "--pipeline", pipeline] + (["--dump-align", dump] if pipeline == "align" else []),
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
    assert line["scaling"] == "strong" and line["n_gpus"] == 1 and line["config"]["utterances"] == n
    assert line["value"] > 0 and line["decode_tokens_per_s"] > 0 and line["config"]["queue"] == queue
    if pipeline == "align":
        assert line["aligned_rank0"] == n
        _check_dumped_alignment(json.load(open(dump)))
    if queue == "dynamic":
        st = line["rank0_stream"]
        assert st["clips"] == n and 0 < st["slot_utilisation"] <= 1


def test_probe_stride_samples_steps(gpu, tiny_gguf):
    """the bench's roofline probe (qasr_set_probe) with probe_stride = 4 times
    every 4th decode step only (HIP events and the device-clock record), and
    the whole-step graph replays in between give the same tokens"""
    m = qasr.Model(tiny_gguf)
    c = qasr.Context(m, max_batch=1, max_ctx=256)
    try:
        pcm = qasr.synth_pcm(7700, 2 * 16000)
        ref = c.transcribe([pcm], max_tokens=13, ignore_eos=True).tokens
        c.set_option("probe_stride", 4)
        assert c.get_option("probe_stride") == 4
        c.set_probe(2)
        got = c.transcribe([pcm], max_tokens=13, ignore_eos=True).tokens
        ms, n, nbytes = c.get_probe()
        c.set_probe(0)
    finally:
        c.close()
        m.close()
    assert got == ref
    assert n == 3 and ms > 0 and nbytes > 0   # decode steps 0, 4, 8 of the 12


def _check_dumped_alignment(d):
    """the driver's document = its classes LIS-repaired x 80 ms; those classes
    = the oracle's wherever the oracle's own margin is clear"""
    import oracle_py as op
    pcm = qasr.synth_pcm(d["seed"], d["n_samples"])
    am = qasr.Model(d["aligner_model"])
    try:
        ids, nw = am.align_tokenize(d["text"])
    finally:
        am.close()
    words, cls = d["doc"]["words"], d["classes"]
    assert [w["word"] for w in words] == d["text"].split() and len(words) == nw and len(cls) == 2 * nw
    dur = np.float32(len(pcm) / SR)
    ts = [float(min(np.float32(k) * np.float32(0.08), dur)) for k in qasr.fix_timestamps(cls)]
    assert [v for w in words for v in (w["start"], w["end"])] == pytest.approx(ts, abs=5e-4)
    op.set_threads(min(16, os.cpu_count() or 1))
    ocls, olg, _ = op.OracleModel(d["aligner_model"]).align_classes(pcm, ids)
    srt = np.sort(olg, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 5e-3 * float(np.abs(olg).max())
    same = np.array(cls) == np.array(ocls)
    assert same[clear].all(), (cls, list(ocls), clear)


def test_engine_after_torch_rccl_in_one_process(tmp_path):
    """bench.py's N > 1 order: torch's HIP runtime and a one-rank RCCL group
    initialised first, then libqasr.so loads (binding to torch's libamdhip64
    by soname) and transcribes -- the multi-GPU bench's control path on one
    GPU.  (The reverse order puts two HSA runtimes in one process.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import os, sys\n"
        f"sys.path.insert(0, {os.path.join(root, 'qwen3-asr.cpp_amd', 'python')!r})\n"
        "import torch, torch.distributed as dist\n"
        "os.environ['MASTER_ADDR'] = '127.0.0.1'; os.environ['MASTER_PORT'] = '29581'\n"
        "torch.cuda.set_device(0)\n"
        "dist.init_process_group('nccl', rank=0, world_size=1); dist.barrier()\n"
        "import qasr\n"
        f"p = {str(tmp_path / 'tiny.gguf')!r}\n"
        "qasr.write_synthetic_gguf(p, 'tiny', 42, 1)\n"
        "m = qasr.Model(p, 0); c = qasr.Context(m, max_batch=1, max_ctx=256)\n"
        "r = c.transcribe([qasr.synth_pcm(5, 16000)], max_tokens=4, ignore_eos=True)\n"
        "t = torch.tensor([float(len(r.tokens[0]))], device='cuda:0'); dist.all_reduce(t)\n"
        "print('ok', int(t.item()))\n"
        "c.close(); m.close(); dist.destroy_process_group()\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and "ok 4" in out.stdout, (out.stdout[-800:], out.stderr[-1500:])
