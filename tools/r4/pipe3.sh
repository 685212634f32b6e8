# fx_pipe v2 (cheap no-record weights path, buffer-descriptor V loads): micro, bench, layer trace
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "1370 2 1" "1370 6 1"; do
  timeout -k 5 60 tools/micro/chain_pipe $a >> gpurun_out/p3_micro.log 2>&1; rc=$?
  [ $rc -gt 1 ] && { echo "micro rc=$rc"; cat gpurun_out/p3_micro.log; exit $rc; }
done
cat gpurun_out/p3_micro.log
fp=1
QASR_FX_PIPE=$fp timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p3_b$fp.log 2>&1 || { tail -5 gpurun_out/p3_b$fp.log; exit 1; }
grep '^{' gpurun_out/p3_b$fp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fx_pipe', $fp, d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
QASR_FX_PIPE=$fp QASR_DEV_TRACE=gpurun_out/p3_tr$fp.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/p3_trb$fp.log 2>&1 || { tail -5 gpurun_out/p3_trb$fp.log; exit 1; }
python3 tools/trace_report.py gpurun_out/p3_tr$fp.bin 2>&1 | head -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_aligner.py -x -v --timeout 300 --timeout-method thread > gpurun_out/p3_t.log 2>&1; rc=$?
tail -3 gpurun_out/p3_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/p3_t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline align --no-probe > gpurun_out/p3_align.log 2>&1 || { tail -5 gpurun_out/p3_align.log; exit 1; }
grep '^{' gpurun_out/p3_align.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('align', d['value'], d['stage_ms_per_step_rank0'])"
