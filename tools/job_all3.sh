#!/bin/bash
# GPU tests + default, batch-64 and align bench lines
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python -u bench.py --no-cpu-baseline
step f16_b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step c4_align 300 python -u bench.py --pipeline align --steps 2 --warmup 1 --no-cpu-baseline --no-probe
