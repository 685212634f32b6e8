#!/bin/bash
# bench lines for the non-headline BASELINE configs (configs[2]/[4], and a
# 64-clip f16 batch) -- reported in DESIGN.md, not the driver's bench line
source ./gpurun_job.sh
export TMPDIR=/tmp
step c2_q8_b64 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step f16_b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe
step c4_align 300 python -u bench.py --pipeline align --steps 2 --warmup 1 --no-cpu-baseline --no-probe
