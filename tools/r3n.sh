# hybrid slow path in the fused chain: parity tests, bench x2, trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 280 --timeout-method thread -k "fused or position_zero or configs1" > gpurun_out/r3n_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3n_t.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3n_b$i.log 2>&1 || exit 1
grep '^{' gpurun_out/r3n_b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('hybrid', d['value'], d['stage_ms_per_step_rank0']['decode'])"
done
QASR_DEV_TRACE=gpurun_out/r3n_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3n_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3n_tr.bin
