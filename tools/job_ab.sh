#!/bin/bash
# A/B: fused vs unfused decode layer (qasr-bench + one-layer trace each)
source ./gpurun_job.sh
export TMPDIR=/tmp
for F in 1 0; do
  QASR_FUSED=$F step bench_f$F 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 3 --warmup 1
  QASR_FUSED=$F QASR_DEV_TRACE=gpurun_out/trace_f$F.bin step trace_f$F 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 1
  python3 tools/trace_report.py gpurun_out/trace_f$F.bin
done
