# fx_pipe (weights one buffer ahead, SGPR operands): micro, parity tests, bench
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "1370 2" "1370 0.5" "1370 8" "600 2" "2000 2"; do
  timeout -k 5 60 tools/micro/chain_pipe $a >> gpurun_out/p1_micro.log 2>&1; rc=$?
  [ $rc -gt 1 ] && { echo "micro rc=$rc"; cat gpurun_out/p1_micro.log; exit $rc; }
done
cat gpurun_out/p1_micro.log
QASR_FX_PIPE=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_batch.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fused or configs1 or fx_seq or batch or teacher or transcribe" > gpurun_out/p1_t.log 2>&1; rc=$?
tail -3 gpurun_out/p1_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/p1_t.log | head -20; exit $rc; }
QASR_FX_PIPE=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p1_b.log 2>&1 || { tail -5 gpurun_out/p1_b.log; exit 1; }
grep '^{' gpurun_out/p1_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
