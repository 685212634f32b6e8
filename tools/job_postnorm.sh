#!/bin/bash
# decode batches: RMS norms fused into the o / down projections (post_norm) vs separate launches
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_q8.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pn_t.log 2>&1
rc=$?; tail -3 gpurun_out/pn_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "batch or configs2" > gpurun_out/pn_t2.log 2>&1
rc=$?; tail -3 gpurun_out/pn_t2.log; [ $rc -ne 0 ] && exit $rc
for pn in 1 0; do
  for q in "" "--q8"; do
    QASR_POST_NORM=$pn timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe $q > gpurun_out/pn_b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pn_b.log') if l.startswith('{')][-1]); print('post_norm=$pn $q', d['value'], d['stage_ms_per_step_rank0']['decode'])"
  done
done
