#!/bin/bash
source ./gpurun_job.sh
export TMPDIR=/tmp
for d in 5 12 20 30 40; do
  QASR_FUSE_ODELAY=$d step native_o$d 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 3 --warmup 1
done
QASR_FUSE_O=0 step native_nofuse 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 3 --warmup 1
