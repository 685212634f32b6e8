#!/bin/bash
source ./gpurun_job.sh
export TMPDIR=/tmp
step b64a 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step b64b 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
