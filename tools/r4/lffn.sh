# FFN joined to the batch-1 attention launch: parity (fused == separate incl. lffn=0, configs[1]), bench, trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fused or configs1 or teacher or prefill_and_steps or position_zero or two_threads" > gpurun_out/lf_t.log 2>&1; rc=$?
tail -3 gpurun_out/lf_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/lf_t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/lf_b.log 2>&1 || { tail -5 gpurun_out/lf_b.log; exit 1; }
grep '^{' gpurun_out/lf_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lffn', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
QASR_LFFN=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/lf_b0.log 2>&1 || { tail -5 gpurun_out/lf_b0.log; exit 1; }
grep '^{' gpurun_out/lf_b0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lffn=0', d['value'], d['stage_ms_per_step_rank0'])"
QASR_DEV_TRACE=gpurun_out/lf_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/lf_trb.log 2>&1 || { tail -5 gpurun_out/lf_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/lf_tr.bin 2>&1 | head -14
exit 0
