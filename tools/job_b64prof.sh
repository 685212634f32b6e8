#!/bin/bash
# kernel-time breakdown of the batched configs (f16 and Q8_0, 64 x 30 s), decode eager
export TMPDIR=/tmp
mkdir -p gpurun_out
export QASR_NO_GRAPH=1
for q in "" "--q8"; do
  n=b64${q:+_q8}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$n -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline --no-probe $q > gpurun_out/$n.log 2>&1 || { echo "fail $n"; exit 1; }
  python3 - gpurun_out/$n/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:100]}")
PY
done
