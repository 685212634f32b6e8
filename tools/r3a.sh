export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a_t.log 2>&1; rc=$?; tail -4 gpurun_out/r3a_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3a_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3a_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'])"
