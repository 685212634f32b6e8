#!/bin/bash
# one rocprofv3 kernel-stats pass over bench.py $BENCH_ARGS (eager decode)
source ./gpurun_job.sh
export TMPDIR=/tmp QASR_NO_GRAPH=1
OUT=${PROF_OUT:-gpurun_out/stats}
step stats 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe $BENCH_ARGS
python3 tools/prof_report.py $OUT > $OUT/summary.json
