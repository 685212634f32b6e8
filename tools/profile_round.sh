#!/bin/bash
# Round-end measurement evidence -> $PROF_OUT (default gpurun_out/prof), copied
# to profiles/<round>/ by hand:
#   bench.json      the default bench.py line (configs[1])
#   configs/*.json  the other BASELINE configs' lines (PROF_CONFIGS=1)
#   stats/          rocprofv3 --kernel-trace --stats over bench.py (decode step
#                   eager, QASR_NO_GRAPH=1: rocprofv3 7.2 faults inside
#                   hipGraphLaunch); its qkv_attn1_kernel average is what the
#                   bench line's roofline probe times with HIP events
#   fetch/ write/   PMC passes (FETCH_SIZE and WRITE_SIZE cannot share one:
#                   MI355X_MICROARCH.md) over qasr-bench, the same workload as
#                   a native program, decode kernels only, 46-token budget
#                   (rocprofv3 --pmc faults under a ctypes-driven process and
#                   after many thousands of counted dispatches)
#   mfma/           PMC pass over the encoder / prefill MFMA kernels:
#                   SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_*, GRBM_GUI_ACTIVE
#   summary.json    tools/prof_report.py
# Every GPU step has its own time limit; the script stops at the first crash
# or timeout and never retries a GPU step.
set -u
OUT=${PROF_OUT:-gpurun_out/prof}
ARGS=${BENCH_ARGS:-}
export TMPDIR=/tmp
mkdir -p "$OUT" gpurun_out
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 to=$2; shift 2
    echo "=== $name" >&2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" >&2
    tail -3 "gpurun_out/$name.log" >&2
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
step bench 600 python -u bench.py $ARGS
grep '^{"metric"' gpurun_out/bench.log > "$OUT/bench.json"
if [ "${PROF_CONFIGS:-0}" = 1 ]; then
    mkdir -p "$OUT/configs"
    step c2_q8_b64 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline
    step f16_b64 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline
    step c4_align 300 python -u bench.py --pipeline align --steps 2 --warmup 1 --no-cpu-baseline
    for f in c2_q8_b64 f16_b64 c4_align; do grep '^{"metric"' gpurun_out/$f.log > "$OUT/configs/$f.json"; done
fi
export QASR_NO_GRAPH=1
step prof_stats 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS
DEC="gemv|qkv_attn1|ffn1|decode_attn"
step prof_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$DEC" -f csv -d "$OUT/fetch" -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.5 $ARGS
step prof_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$DEC" -f csv -d "$OUT/write" -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.5 $ARGS
ENC="gemm_kernel|gemm_glds|gemm8p|gemm_q8|enc_attn|prefill_attn|conv1"
step prof_mfma 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_I8 GRBM_GUI_ACTIVE --kernel-include-regex "$ENC" -f csv -d "$OUT/mfma" -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.05 $ARGS
python3 tools/prof_report.py "$OUT" > "$OUT/summary.json"
