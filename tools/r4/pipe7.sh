# fx_pipe = 3: single-wave chain workgroups on the default weights path: bench + trace, parity (fused == separate, configs[1])
export TMPDIR=/tmp
mkdir -p gpurun_out

QASR_FX_PIPE=3 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p7_b.log 2>&1 || { tail -5 gpurun_out/p7_b.log; exit 1; }
grep '^{' gpurun_out/p7_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fx3', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
QASR_FX_PIPE=3 QASR_DEV_TRACE=gpurun_out/p7_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/p7_trb.log 2>&1 || { tail -5 gpurun_out/p7_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/p7_tr.bin 2>&1 | head -12
QASR_FX_PIPE=3 timeout -k 10 700 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fused or configs1 or teacher or prefill_and_steps" > gpurun_out/p7_t.log 2>&1; rc=$?
tail -3 gpurun_out/p7_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/p7_t.log | head -20; exit $rc; }
exit 0
