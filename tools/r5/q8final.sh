# round-5 Q8_0 decode-batch profile after the decode-batch changes (tools/profile_batch.sh),
# written under gpurun_out/ and copied to profiles/r5/batch/q8 afterwards (the configs[2]
# line: gpurun_out/c2_q8_b64.log of the previous form of this script)
export TMPDIR=/tmp
mkdir -p gpurun_out
PROF_BATCH_CFGS=q8 PROF_OUT=gpurun_out/r5q8batch bash tools/profile_batch.sh
