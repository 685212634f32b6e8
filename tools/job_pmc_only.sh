#!/bin/bash
source ./gpurun_job.sh
export TMPDIR=/tmp QASR_NO_GRAPH=1
OUT=${PROF_OUT:-gpurun_out/prof}
RX=${PMC_REGEX:-gemv_kernel}
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $OUT/fetch -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.5
step prof_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $OUT/write -o run -- ./qwen3-asr.cpp_amd/qasr-bench --steps 1 --warmup 0 --tok-rate 0.5
python3 tools/prof_report.py $OUT > $OUT/summary.json
