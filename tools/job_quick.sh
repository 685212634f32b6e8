#!/bin/bash
# quick GPU iteration: parity tests, bench (no CPU leg), one-layer dev trace
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-}
QASR_DEV_TRACE=gpurun_out/trace.bin step trace 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 1
python3 tools/trace_report.py gpurun_out/trace.bin
