# round-5 final evidence with the final code: tools/profile_round.sh (default bench line,
# the other configs' lines, kernel-trace stats, FETCH / WRITE / MFMA passes, summary)
# into gpurun_out/r5final, copied into profiles/r5/ afterwards
export TMPDIR=/tmp
PROF_OUT=gpurun_out/r5final PROF_CONFIGS=1 bash tools/profile_round.sh
# keep the merge-back under gpurun's 64 MiB: the per-dispatch kernel traces stay on the box
find gpurun_out/r5final -name "*kernel_trace.csv" -delete
du -sh gpurun_out/r5final
