# per-8-key slow path in the fused chain: microbench, parity tests, bench A/B (ffn_in off)
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in "0 4 0" "0 4 0x10" "0 4 0x1010101" "5 4 0" "5 4 0x1" "5 4 0x100000001"; do timeout -k 5 30 ./tools/micro/chain_role $m || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 280 --timeout-method thread -k "fused or position_zero or configs1" > gpurun_out/r3m_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3m_t.log; [ $rc -ne 0 ] && exit $rc
QASR_FFN_IN=0 timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3m_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3m_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('mask', d['value'], d['stage_ms_per_step_rank0']['decode'])"
QASR_FFN_IN=0 QASR_DEV_TRACE=gpurun_out/r3m_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3m_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3m_tr.bin
