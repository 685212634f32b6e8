#!/bin/bash
# fused batch-1 FFN: down-weight delay x poll delay sweep against the unfused launches
source ./gpurun_job.sh
export TMPDIR=/tmp
QASR_FUSE_FFN=0 step bench_off 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
for w in 6 10 14 18; do for d in 0 4; do QASR_FFN_WDELAY=$w QASR_FFN_DELAY=$d step bench_w${w}_d$d 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2; done; done
QASR_FFN_WDELAY=${TW:-10} QASR_DEV_TRACE=gpurun_out/trace.bin step trace 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 1
python3 tools/trace_report.py gpurun_out/trace.bin
