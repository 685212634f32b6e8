#!/bin/bash
# same-box A/B of the gemm8p epilogue without per-store waits in the 64 x 30 s line and the set:
# base = tools/r6/libbase/libqasr.so (HEAD epilogue), new = the in-tree library
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/g35.txt
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export QASR_LIB_OVERRIDE=$PWD/tools/r6/libbase/libqasr.so; else unset QASR_LIB_OVERRIDE; fi
    timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g35_$v.json 2> gpurun_out/g35.err || { tail gpurun_out/g35.err; exit 1; }
    python3 -c "
import json
d = json.load(open('gpurun_out/g35_$v.json')); u = d.get('utterance_set') or {}
print('$v', d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" | tee -a gpurun_out/g35.txt
  done
done
