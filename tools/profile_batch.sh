#!/bin/bash
# Decode-batch counters: per config (f16 / Q8_0, 64 x 30 s; PROF_BATCH=128: 128 x 30 s)
#   $OUT/<cfg>/stats   rocprofv3 --kernel-trace --stats over bench.py (eager decode, QASR_NO_GRAPH=1; one
#                      warm-up step first, so first-call costs stay out: the round-3 Q8 conv1 figure)
#   $OUT/<cfg>/fetch   FETCH_SIZE over qasr-bench, decode-batch kernels only
#   $OUT/<cfg>/write   WRITE_SIZE, same
#   $OUT/<cfg>/mfma    MFMA busy / ops, same
#   $OUT/<cfg>/summary.json   tools/prof_report.py
# each GPU step has its own time limit; the script stops at the first failure
set -u
OUT=${PROF_OUT:-gpurun_out/prof_batch}
export TMPDIR=/tmp
mkdir -p "$OUT" gpurun_out
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 to=$2; shift 2
    echo "=== $name" >&2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" >&2
    tail -2 "gpurun_out/$name.log" >&2
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
DEC="gemm_skinny|decode_attn|lmhead|rmsnorm|gemv"
for cfg in ${PROF_BATCH_CFGS:-f16 q8}; do
    Q=""; [ "$cfg" = q8 ] && Q="--q8"
    D="$OUT/$cfg"; mkdir -p "$D"
    step pb_${cfg}_line 300 python -u bench.py $Q --batch ${PROF_BATCH:-64} --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --set-utterances 0
    grep '^{"metric"' gpurun_out/pb_${cfg}_line.log > "$D/bench.json"
    QASR_NO_GRAPH=1 step pb_${cfg}_stats 300 rocprofv3 --kernel-trace --stats -f csv -d "$D/stats" -o run -- python3 bench.py $Q --batch ${PROF_BATCH:-64} --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 0.5 --set-utterances 0
    step pb_${cfg}_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$DEC" -f csv -d "$D/fetch" -o run -- ./qwen3-asr.cpp_amd/qasr-bench $Q --batch ${PROF_BATCH:-64} --seconds 30 --steps 1 --warmup 0 --tok-rate 0.2
    step pb_${cfg}_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$DEC" -f csv -d "$D/write" -o run -- ./qwen3-asr.cpp_amd/qasr-bench $Q --batch ${PROF_BATCH:-64} --seconds 30 --steps 1 --warmup 0 --tok-rate 0.2
    step pb_${cfg}_mfma 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_I8 GRBM_GUI_ACTIVE --kernel-include-regex "$DEC" -f csv -d "$D/mfma" -o run -- ./qwen3-asr.cpp_amd/qasr-bench $Q --batch ${PROF_BATCH:-64} --seconds 30 --steps 1 --warmup 0 --tok-rate 0.2
    python3 tools/prof_report.py "$D" > "$D/summary.json"
done
