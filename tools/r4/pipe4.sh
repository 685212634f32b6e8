# fx_pipe = 2 (split-side weights): parity (fused == separate, configs[1] full), bench, layer trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 60 tools/micro/chain_pipe 1370 2 1 > gpurun_out/p4_micro.log 2>&1; rc=$?; cat gpurun_out/p4_micro.log; [ $rc -gt 1 ] && exit $rc
QASR_FX_PIPE=2 timeout -k 10 700 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_batch.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fused or configs1 or batch or teacher or transcribe or prefill_and_steps" > gpurun_out/p4_t.log 2>&1; rc=$?
tail -3 gpurun_out/p4_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/p4_t.log | head -20; exit $rc; }
cp gpurun_out/parity.json gpurun_out/p4_parity.json
for fp in 2; do
QASR_FX_PIPE=$fp timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p4_b$fp.log 2>&1 || { tail -5 gpurun_out/p4_b$fp.log; exit 1; }
grep '^{' gpurun_out/p4_b$fp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fx_pipe', $fp, d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
QASR_FX_PIPE=$fp QASR_DEV_TRACE=gpurun_out/p4_tr$fp.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/p4_trb$fp.log 2>&1 || { tail -5 gpurun_out/p4_trb$fp.log; exit 1; }
python3 tools/trace_report.py gpurun_out/p4_tr$fp.bin 2>&1 | head -12
done
