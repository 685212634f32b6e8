# round-3 evidence: full GPU suite, smoke, default bench line (with the CPU baseline)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread > gpurun_out/final_t.log 2>&1; rc=$?; tail -3 gpurun_out/final_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/final_t.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
grep '^{' gpurun_out/final_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['cpu_baseline'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
