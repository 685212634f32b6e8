#!/bin/bash
# round-end evidence: default bench line (with CPU baseline), the non-default
# config lines, rocprofv3 stats + PMC passes -> $PROF_OUT (copied to profiles/)
source ./gpurun_job.sh
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT/configs
step bench 600 python -u bench.py
grep '^{"metric"' gpurun_out/bench.log > $OUT/bench.json
step c2_q8_b64 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step f16_b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step c4_align 300 python -u bench.py --pipeline align --steps 2 --warmup 1 --no-cpu-baseline --no-probe
for f in c2_q8_b64 f16_b64 c4_align; do grep '^{"metric"' gpurun_out/$f.log > $OUT/configs/$f.json; done
PMC_REGEX="gemv|decode_attn" bash tools/job_prof.sh
