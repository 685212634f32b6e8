# Q8_0 skinny GEMMs with every chunk of a wave in flight: tests + configs[2] line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_q8.py tests/test_gpu_full.py -x -q --timeout 580 --timeout-method thread -k "q8 or configs2" > gpurun_out/r3r_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3r_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3r_t.log | head; exit $rc; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3r_b$r.log 2>&1 || exit 1
grep '^{' gpurun_out/r3r_b$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q8', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
