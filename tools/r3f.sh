# fused exact attention after the compact slow path / split weights: parity, bench, layer-14 trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "match_separate or position_zero or configs1" > gpurun_out/r3f_t.log 2>&1; rc=$?; tail -4 gpurun_out/r3f_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3f_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3f_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'], d['decode_attention'][-40:])"
QASR_DEV_TRACE=gpurun_out/r3f_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3f_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3f_tr.bin
for m in "0 4" "0 4 0x10" "2 4" "3 4" "4 4"; do timeout -k 5 30 ./tools/micro/chain_role $m || exit 1; done
