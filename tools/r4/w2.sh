# chain weights two groups ahead + o-proj 2 rows a wave (3 blocks a CU): parity, bench, trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fused or configs1 or teacher or prefill_and_steps or position_zero or two_threads or timeout or long" > gpurun_out/w2_t.log 2>&1; rc=$?
tail -3 gpurun_out/w2_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/w2_t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/w2_b.log 2>&1 || { tail -5 gpurun_out/w2_b.log; exit 1; }
grep '^{' gpurun_out/w2_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
QASR_DEV_TRACE=gpurun_out/w2_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/w2_trb.log 2>&1 || { tail -5 gpurun_out/w2_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/w2_tr.bin 2>&1 | head -12
exit 0
