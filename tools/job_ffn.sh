#!/bin/bash
# fused batch-1 FFN: parity tests, then bench with the fusion off / on and a down-weight delay sweep
source ./gpurun_job.sh
export TMPDIR=/tmp
[ -n "${NO_TESTS:-}" ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
QASR_FUSE_FFN=0 step bench_off 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
step bench_on 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
for d in 0 4 12; do QASR_FFN_DELAY=$d step bench_d$d 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2; done
QASR_DEV_TRACE=gpurun_out/trace.bin step trace 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 1
python3 tools/trace_report.py gpurun_out/trace.bin
