# batch exact decode chain with 4 V^T register buffers (3 in flight): parity, B=64 f16 / Q8 benches
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py tests/test_gpu_q8.py -x -q --timeout 600 --timeout-method thread -k "fx_seq or configs3 or batch or separate or teacher or q8" > gpurun_out/vn_t.log 2>&1; rc=$?
tail -3 gpurun_out/vn_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/vn_t.log | head -20; exit $rc; }
for q in "" "--q8"; do
timeout -k 10 300 python -u bench.py $q --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/vn_b$q.log 2>&1 || { tail -5 gpurun_out/vn_b$q.log; exit 1; }
grep '^{' gpurun_out/vn_b$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b64 $q', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']], d['decode_hbm']['frac'])"
done
exit 0
