#!/bin/bash
# decode-batch LM head tilings (TEMP knob QASR_LMH): kernel time from rocprofv3 stats
export TMPDIR=/tmp
mkdir -p gpurun_out
export QASR_NO_GRAPH=1
for v in 0 1 2 3 4; do
  QASR_LMH=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/lmh$v -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > gpurun_out/lmh$v.log 2>&1 || { echo fail $v; exit 1; }
  python3 - gpurun_out/lmh$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'gemm_skinny_kernel' in r['Name'] and ', 3,' in r['Name'].replace(' ', ' '):
        print(sys.argv[2], r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3)
PY
done
