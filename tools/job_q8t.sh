#!/bin/bash
# Q8_0 tiled GEMM tile shapes (TEMP knob QASR_Q8T) on configs[2]
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 0 1 2; do
  QASR_Q8T=$t timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/q8t.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/q8t.log') if l.startswith('{')][-1]); print('q8t=$t', d['value'], d['stage_ms_per_step_rank0'])"
done
