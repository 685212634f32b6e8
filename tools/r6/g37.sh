#!/bin/bash
# batch-1 GEMV bias / residual requested ahead of the stores: GPU suite, then same-box A/B
# (base = tools/r6/libbase/libqasr.so, the previous GEMV) of the driver's bench command, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g37_t.log 2>&1 || { tail -40 gpurun_out/g37_t.log; exit 2; }
tail -3 gpurun_out/g37_t.log
: > gpurun_out/g37.txt
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export QASR_LIB_OVERRIDE=$PWD/tools/r6/libbase/libqasr.so; else unset QASR_LIB_OVERRIDE; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/g37_$v.json 2> gpurun_out/g37.err || { tail gpurun_out/g37.err; exit 4; }
    python3 -c "
import json
d = json.load(open('gpurun_out/g37_$v.json')); u = d.get('utterance_set') or {}
print('$v', d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" >> gpurun_out/g37.txt
  done
done
cat gpurun_out/g37.txt
