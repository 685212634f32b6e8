#!/bin/bash
# default bench line + rocprofv3 stats/PMC passes into $PROF_OUT
source ./gpurun_job.sh
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
step bench 600 python -u bench.py
grep '^{"metric"' gpurun_out/bench.log > $OUT/bench.json
PMC_REGEX="gemv|decode_attn" bash tools/job_prof.sh
