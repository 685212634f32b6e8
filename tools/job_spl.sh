#!/bin/bash
# batch-1 attention split length with the fused launches: 128 (default at >= 1k keys) vs 64
source ./gpurun_job.sh
export TMPDIR=/tmp
for r in a b; do
step spl_def_$r 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
QASR_ATT_SPL1=64 step spl_64_$r 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
done
QASR_ATT_SPL1=64 QASR_DEV_TRACE=gpurun_out/trace.bin step trace 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 1
python3 tools/trace_report.py gpurun_out/trace.bin
