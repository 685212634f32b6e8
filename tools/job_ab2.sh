#!/bin/bash
# GPU tests, then bench lines with and without an env switch ($AB_ENV), batch 64 and default
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
env $AB_ENV bash -c 'source ./gpurun_job.sh; step b64_ab 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe'
step b1 300 python -u bench.py --no-cpu-baseline
env $AB_ENV bash -c 'source ./gpurun_job.sh; step b1_ab 300 python -u bench.py --no-cpu-baseline'
