#!/bin/bash
# rocprofv3 passes for profiles/ (see tools/prof_report.py):
#   1. --kernel-trace --stats over the bench.py command itself (decode step
#      eager, QASR_NO_GRAPH=1: rocprofv3 7.2 faults inside hipGraphLaunch);
#   2. one PMC pass per TCC counter group (MI355X_MICROARCH.md: FETCH_SIZE and
#      WRITE_SIZE cannot share a pass) over qasr-bench, the same workload as a
#      native program, with a 46-token decode budget (rocprofv3 --pmc faults
#      after some thousands of counted dispatches; bytes per launch do not
#      depend on the budget).
source ./gpurun_job.sh
export TMPDIR=/tmp QASR_NO_GRAPH=1
OUT=${PROF_OUT:-gpurun_out/prof}
ARGS=${BENCH_ARGS:-}
RX=${PMC_REGEX:-gemv_kernel}
step prof_stats 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $OUT/fetch -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.5 $ARGS
step prof_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $OUT/write -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.5 $ARGS
python3 tools/prof_report.py $OUT > $OUT/summary.json
