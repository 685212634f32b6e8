# round-6 GPU job 20: the other configs' lines (configs[2] Q8_0 64 x 30 s, f16 64 x 30 s, configs[4] align) and the
# decode-batch counters at 128 slots (tools/profile_batch.sh, f16)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6configs
for spec in "c2_q8_b64:--q8 --batch 64 --seconds 30" "f16_b64:--batch 64 --seconds 30" "c4_align:--pipeline align"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python -u bench.py $a --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$n.log 2>&1 || { tail gpurun_out/$n.log; exit 1; }
  grep '^{"metric"' gpurun_out/$n.log > gpurun_out/r6configs/$n.json
done
PROF_OUT=gpurun_out/r6batch PROF_BATCH=128 PROF_BATCH_CFGS=f16 bash tools/profile_batch.sh
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*agent_info.csv" -delete
du -sh gpurun_out
