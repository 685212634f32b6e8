# decode-batch FFN in one launch: bit-identity, batch tests, 64 x 30 s A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_batch.py tests/test_gpu_stream.py -x -v --timeout 580 --timeout-method thread -k "ffn_batch or batch or configs3 or stream" > gpurun_out/r3v_t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/r3v_t.log | tail -25; tail -3 gpurun_out/r3v_t.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
QASR_FFN_BATCH=$v timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3v_b$v.log 2>&1 || exit 1
grep '^{' gpurun_out/r3v_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ffn_batch=$v', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
