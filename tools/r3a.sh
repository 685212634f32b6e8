# round-3 iteration job: chain microbench, GPU tests, a short bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 60 ./tools/micro/chain_asm > gpurun_out/r3_chain.log 2>&1; cat gpurun_out/r3_chain.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_tf.log 2>&1; rc=$?; tail -15 gpurun_out/r3_tf.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_full.py > gpurun_out/r3_t.log 2>&1; rc=$?; tail -4 gpurun_out/r3_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3_b.log 2>&1 || exit 1
grep '^{' gpurun_out/r3_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['decode_attention'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
