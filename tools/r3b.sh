# round-3 iteration: fused exact attention timing (bench + device trace of layer 14)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 60 ./tools/micro/chain_asm; timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "match_separate or position_zero" > gpurun_out/r3b_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3b_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3b_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3b_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
QASR_DEV_TRACE=gpurun_out/r3b_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3b_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3b_tr.bin
