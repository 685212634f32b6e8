# FFN roles in the batch-1 QKV launch: targeted tests, A/B bench, layer-14 trace; LM head sweep
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/micro/lmh_bench > gpurun_out/r3k_lmh.log 2>&1; rc=$?; cat gpurun_out/r3k_lmh.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_refapi.py -x -v --timeout 280 --timeout-method thread -k "fused or position_zero or configs1 or refapi or reference" > gpurun_out/r3k_t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/r3k_t.log | tail -30; tail -3 gpurun_out/r3k_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3k_b1.log 2>&1 || exit 1
grep '^{' gpurun_out/r3k_b1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ffn_in=1', d['value'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
QASR_FFN_IN=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3k_b0.log 2>&1 || exit 1
grep '^{' gpurun_out/r3k_b0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ffn_in=0', d['value'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
for v in 0 1; do
QASR_FFN_IN=$v QASR_DEV_TRACE=gpurun_out/r3k_tr$v.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3k_tr$v.log 2>&1 || exit 1
echo "trace ffn_in=$v"; python3 tools/trace_report.py gpurun_out/r3k_tr$v.bin
done
