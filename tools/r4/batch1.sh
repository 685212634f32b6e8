# skinny in-flight: bit-identity test, batch benches (f16 and q8_0 64 x 30 s) with skinny_inf 1 / 0
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 300 --timeout-method thread -k "skinny_inflight or configs3" > gpurun_out/b1_t.log 2>&1; rc=$?
tail -3 gpurun_out/b1_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/b1_t.log | head -20; exit $rc; }
for q in "" "--q8"; do for inf in 1 0; do
  QASR_SKINNY_INF=$inf timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --batch 64 --seconds 30 $q > gpurun_out/b1_b$inf$q.log 2>&1 || { tail -5 gpurun_out/b1_b$inf$q.log; exit 1; }
  grep '^{' gpurun_out/b1_b$inf$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inf $inf $q', d['value'], d['stage_ms_per_step_rank0'], d.get('decode_hbm',{}).get('frac'))"
done; done
