#!/bin/bash
# the tiled GEMMs' shared epilogue without per-store waits (gemm_kernel / gemm_glds / gemm_q8):
# GPU suite, then same-box A/B (base = tools/r6/libbase/libqasr.so, the previous epilogue) of
# the Q8_0 64 x 30 s line and the driver's bench command, then the other config lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g36_t.log 2>&1 || { tail -40 gpurun_out/g36_t.log; exit 2; }
tail -3 gpurun_out/g36_t.log
: > gpurun_out/g36.txt
for v in new base; do
  if [ $v = base ]; then export QASR_LIB_OVERRIDE=$PWD/tools/r6/libbase/libqasr.so; else unset QASR_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g36_q8_$v.json 2> gpurun_out/g36.err || { tail gpurun_out/g36.err; exit 3; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/g36_bench_$v.json 2> gpurun_out/g36.err || { tail gpurun_out/g36.err; exit 4; }
  for f in q8 bench; do
    python3 -c "
import json
d = json.load(open('gpurun_out/g36_${f}_$v.json')); u = d.get('utterance_set') or {}
print('${f}_$v', d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" >> gpurun_out/g36.txt
  done
done
unset QASR_LIB_OVERRIDE
for spec in "f16_b64:--batch 64 --seconds 30" "c4_align:--pipeline align"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python -u bench.py $a --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g36_$n.json 2> gpurun_out/g36_$n.err || { tail gpurun_out/g36_$n.err; exit 5; }
  python3 -c "
import json
d = json.load(open('gpurun_out/g36_$n.json')); u = d.get('utterance_set') or {}
print('$n', d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" >> gpurun_out/g36.txt
done
cat gpurun_out/g36.txt
