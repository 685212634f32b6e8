#!/bin/bash
# GPU tests + batch-64 bench lines (f16, q8_0) + the default bench
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step f16_b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step q8_b64 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
[ -n "$WITH_DEFAULT" ] && step bench 300 python -u bench.py --no-cpu-baseline
true
