# decode batches: all chunks of a wave in flight (skinny GEMMs), per-8-key slow path in the batch exact chain
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_q8.py tests/test_gpu_stream.py tests/test_gpu_full.py -x -q --timeout 580 --timeout-method thread -k "not fused and not position_zero and not configs1 and not two_threads and not wait_timeout" > gpurun_out/r3q_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3q_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3q_t.log | head; exit $rc; }
for q in "" "--q8"; do
timeout -k 10 300 python -u bench.py $q --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3q_b$q.log 2>&1 || exit 1
grep '^{' gpurun_out/r3q_b$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$q', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
