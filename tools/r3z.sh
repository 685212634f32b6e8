# one-launch exact batch attention with the V^T prefix copied into LDS (fx_seq 2) vs 1: bit-identity, A/B at 64 x 30 s
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_batch.py -x -v --timeout 580 --timeout-method thread -k "fx_seq or configs3 or batch64 or decode_batch" > gpurun_out/r3z_t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/r3z_t.log | tail -20; tail -3 gpurun_out/r3z_t.log; [ $rc -ne 0 ] && exit $rc
for v in 2 1 2 1; do
QASR_FX_SEQ=$v timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3z_b$v.log 2>&1 || exit 1
grep '^{' gpurun_out/r3z_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fx_seq=$v', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
QASR_FX_SEQ=2 timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3z_q8.log 2>&1 || exit 1
grep '^{' gpurun_out/r3z_q8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q8 fx_seq=2', d['value'], d['stage_ms_per_step_rank0'])"
