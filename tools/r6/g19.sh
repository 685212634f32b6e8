# round-6 GPU job 19: the round's evidence (tools/profile_round.sh: bench line, rocprofv3 kernel trace --stats,
# FETCH / WRITE / MFMA PMC passes, summary.json) into gpurun_out/r6prof; the raw per-dispatch traces are dropped
# after the summary (gpurun returns at most 64 MiB)
PROF_OUT=gpurun_out/r6prof PROF_CONFIGS=0 bash tools/profile_round.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*agent_info.csv" -delete
du -sh gpurun_out
