#!/bin/bash
# GPU tests + default bench (no CPU leg), optional env A/B of the bench
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python -u bench.py --no-cpu-baseline
[ -n "$AB_ENV" ] && env $AB_ENV bash -c 'source ./gpurun_job.sh; step bench_ab 300 python -u bench.py --no-cpu-baseline'
true
