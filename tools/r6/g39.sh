#!/bin/bash
# layernorm weights / bias requested with x (no load between its stores): GPU suite, 64 x 30 s line, bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g39_t.log 2>&1 || { tail -40 gpurun_out/g39_t.log; exit 2; }
tail -3 gpurun_out/g39_t.log
: > gpurun_out/g39.txt
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g39_b64.json 2> gpurun_out/g39.err || { tail gpurun_out/g39.err; exit 3; }
timeout -k 10 300 python -u bench.py > gpurun_out/g39_bench.json 2> gpurun_out/g39.err || { tail gpurun_out/g39.err; exit 4; }
python3 -c "
import json
for f in ('g39_b64', 'g39_bench'):
    d = json.load(open('gpurun_out/%s.json' % f)); u = d.get('utterance_set') or {}
    print(f, d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" | tee gpurun_out/g39.txt
