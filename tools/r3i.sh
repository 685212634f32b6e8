# LM head one-launch microbench, full -m gpu suite, default bench + f16 B=64 line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/lmh_bench > gpurun_out/r3i_lmh.log 2>&1; rc=$?; cat gpurun_out/r3i_lmh.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread > gpurun_out/r3i_t.log 2>&1; rc=$?; grep -E "FAIL|ERROR" gpurun_out/r3i_t.log | head; tail -3 gpurun_out/r3i_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3i_s.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3i_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3i_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['decode_attention'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3i_b64.log 2>&1 || exit 1
grep '^{' gpurun_out/r3i_b64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d.get('decode_hbm'))"
