#!/bin/bash
# fused batch-1 FFN: finer sweep around the best down-weight delay, repeated
source ./gpurun_job.sh
export TMPDIR=/tmp
QASR_FUSE_FFN=0 step bench_off 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
for c in 14_4 12_4 16_4 14_2 14_6 14_4 16_6 20_6 14_4; do w=${c%_*}; d=${c#*_}; QASR_FFN_WDELAY=$w QASR_FFN_DELAY=$d step b_${c} 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2; done
QASR_FUSE_FFN=0 step bench_off2 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
