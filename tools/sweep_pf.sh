#!/bin/bash
# Infinity Cache prefetch role of the batch-1 QKV launch: decode ms of the 92 s clip per (blocks, delay)
set -u
for cfg in "0 0" "128 30" "128 40" "256 30" "128 50" "64 35"; do
    set -- $cfg
    out=$(QASR_PF_BLOCKS=$1 QASR_PF_DELAY=$2 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe 2>/dev/null | grep '^{"metric"') || exit 1
    echo "pf=$1 delay=$2 $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms_per_step_rank0"]["decode"])')"
done
