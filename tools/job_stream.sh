#!/bin/bash
# streamed batch attention splits (att_stream) vs one workgroup per split
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_q8.py -x -q --timeout 240 --timeout-method thread > gpurun_out/st_t.log 2>&1
rc=$?; tail -3 gpurun_out/st_t.log; [ $rc -ne 0 ] && exit $rc
for st in 1 0; do
  for q in "" "--q8"; do
    QASR_ATT_STREAM=$st timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline $q > gpurun_out/st_b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/st_b.log') if l.startswith('{')][-1]); print('stream=$st $q', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'])"
  done
done
