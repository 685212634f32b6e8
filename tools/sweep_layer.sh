#!/bin/bash
# delay sweep of the batch-1 layer launch (decode ms of the 92 s clip per setting)
set -u
for cfg in "0 30 8" "16 30 8" "32 40 8" "48 60 8" "24 24 4" "64 80 8" "100 120 8"; do
    set -- $cfg
    out=$(QASR_GU_DELAY=$1 QASR_DN_WDELAY=$2 QASR_DN_DELAY=$3 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe 2>/dev/null | grep '^{"metric"') || exit 1
    echo "gu=$1 dnw=$2 dnd=$3 $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms_per_step_rank0"]["decode"])')"
done
out=$(QASR_FUSE_LAYER=0 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe 2>/dev/null | grep '^{"metric"') || exit 1
echo "two-launch $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms_per_step_rank0"]["decode"])')"
