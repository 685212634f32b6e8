# LM head (WPG, D) sweep, refapi tests, smoke, default bench, batch counters
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/micro/lmh_bench > gpurun_out/r3j_lmh.log 2>&1; rc=$?; cat gpurun_out/r3j_lmh.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_refapi.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/r3j_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3j_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3j_s.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3j_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3j_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['decode_attention'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['cpu_baseline']['value'])"
bash tools/profile_batch.sh
