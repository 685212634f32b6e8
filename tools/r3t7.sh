# chain weight phase weights by v_readlane from one VGPR per buffer: trace, fused-launch tests, configs[1] lines
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_DEV_TRACE=gpurun_out/r3t7_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3t7_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3t7_tr.bin
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 580 --timeout-method thread -k "fused or position_zero or configs1" > gpurun_out/r3t7_t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/r3t7_t.log | tail -12; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3t7_b$i.log 2>&1 || exit 1
grep '^{' gpurun_out/r3t7_b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
