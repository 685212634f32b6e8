# decode-batch counters at 128 rows (the utterance set's slots per context): tools/profile_batch.sh
# with PROF_BATCH=128 into gpurun_out/r5b128, copied to profiles/r5/batch128 afterwards
export TMPDIR=/tmp
PROF_BATCH=128 PROF_OUT=gpurun_out/r5b128 bash tools/profile_batch.sh || exit 1
find gpurun_out/r5b128 -name "*kernel_trace.csv" -delete
du -sh gpurun_out/r5b128
