#!/bin/bash
# GPU tests + batch-64 bench lines (attention split A/B) + the default bench
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step f16_b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
QASR_ATT_SPL=128 step f16_b64_s128 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step bench 300 python -u bench.py --no-cpu-baseline
