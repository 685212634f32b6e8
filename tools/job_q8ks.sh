#!/bin/bash
# Q8_0 tiled GEMM K-stage depth (prefill / encoder of configs[2]) + post_norm bit-identity test
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ks_t.log 2>&1
rc=$?; tail -3 gpurun_out/ks_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/ks_b.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ks_b.log') if l.startswith('{')][-1]); print('q8 b64', d['value'], d['stage_ms_per_step_rank0'])"
