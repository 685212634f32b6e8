# round-3 re-entry check: full -m gpu suite, smoke, default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread > gpurun_out/r3h_t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|SKIP" gpurun_out/r3h_t.log | tail -120; tail -3 gpurun_out/r3h_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3h_s.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3h_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3h_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['decode_attention'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['cpu_baseline']['value'])"
