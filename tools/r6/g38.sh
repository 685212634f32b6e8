#!/bin/bash
# round-6 final evidence after the GEMM epilogue fixes: the default bench line with its rocprof / PMC
# passes (tools/profile_round.sh), then the decode-batch counters at 128 slots (tools/profile_batch.sh, f16)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r6prof gpurun_out/r6batch
PROF_OUT=gpurun_out/r6prof PROF_CONFIGS=0 bash tools/profile_round.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*agent_info.csv" -delete
PROF_OUT=gpurun_out/r6batch PROF_BATCH=128 PROF_BATCH_CFGS=f16 bash tools/profile_batch.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*agent_info.csv" -delete
