#!/bin/bash
# persistent-grid wide projections: micro A/B, the GPU suite, the 64 x 30 s line and the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o /tmp/g8_bench tools/micro/g8_bench.hip > gpurun_out/g31_build.txt 2>&1 || exit 1
timeout -k 10 300 /tmp/g8_bench > gpurun_out/g31_g8.txt 2>&1 || { tail gpurun_out/g31_g8.txt; exit 1; }
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g31_t.log 2>&1 || { tail -40 gpurun_out/g31_t.log; exit 2; }
tail -3 gpurun_out/g31_t.log
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g31_b64.json 2> gpurun_out/g31_b64.err || { tail gpurun_out/g31_b64.err; exit 3; }
timeout -k 10 300 python -u bench.py > gpurun_out/g31_bench.json 2> gpurun_out/g31_bench.err || { tail gpurun_out/g31_bench.err; exit 4; }
python3 -c "
import json
for f in ('g31_b64', 'g31_bench'):
    d = json.load(open('gpurun_out/%s.json' % f)); u = d.get('utterance_set') or {}
    print(f, d['value'], d['stage_ms_per_step_rank0'], u.get('value'), (u.get('ragged') or {}).get('value'))
" | tee gpurun_out/g31.txt
