#!/bin/bash
# same-box A/B: 64 x 30 s line with 4 vs 8 HIP hardware queues
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/g33.txt
for rep in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/r6/hwq_ab.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g33_$q.json 2> gpurun_out/g33.err || { tail gpurun_out/g33.err; exit 1; }
    python3 -c "
import json
d = json.load(open('gpurun_out/g33_$q.json')); u = d.get('utterance_set') or {}
print('hwq$q', d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" >> gpurun_out/g33.txt
  done
done
