#!/bin/bash
# exact decode chain with 128-key V buffers: Q8_0 tests, configs[1] full test (both decode modes), configs[2] line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dxq_t.log 2>&1
rc=$?; tail -2 gpurun_out/dxq_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "configs1 or configs2" > gpurun_out/dxq_t2.log 2>&1
rc=$?; tail -2 gpurun_out/dxq_t2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dxq_b.log 2>&1 || exit 1
grep "^{" gpurun_out/dxq_b.log > gpurun_out/dxq_c2.json
python3 -c "import json; d=json.load(open('gpurun_out/dxq_c2.json')); print('q8 b64', d['value'], d['stage_ms_per_step_rank0'])"
