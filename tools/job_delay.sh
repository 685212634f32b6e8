#!/bin/bash
source ./gpurun_job.sh
export TMPDIR=/tmp
for d in 10 14 18 24; do
  QASR_FUSE_DELAY=$d step native_d$d 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 3 --warmup 1
done
