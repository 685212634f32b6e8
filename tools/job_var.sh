#!/bin/bash
# variance check: bench.py with and without the LM-head probe, native qasr-bench
source ./gpurun_job.sh
export TMPDIR=/tmp
step b_probe 300 python -u bench.py --no-cpu-baseline
step b_noprobe 300 python -u bench.py --no-cpu-baseline --no-probe
step native 120 ./qwen3-asr.cpp_amd/qasr-bench --steps 3 --warmup 1
step b_probe2 300 python -u bench.py --no-cpu-baseline
