#!/bin/bash
# default bench with and without an env switch ($AB_ENV)
source ./gpurun_job.sh
export TMPDIR=/tmp
step b1 300 python -u bench.py --no-cpu-baseline
env $AB_ENV bash -c 'source ./gpurun_job.sh; step b1_ab 300 python -u bench.py --no-cpu-baseline'
step b1_again 300 python -u bench.py --no-cpu-baseline
