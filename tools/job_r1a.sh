#!/bin/bash
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 300 python -u bench.py
step prof_bench 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
find gpurun_out/prof_bench -name '*stats*'
