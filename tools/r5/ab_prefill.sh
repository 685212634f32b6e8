# same-box A/B of the f16 64 x 30 s line: this tree's libqasr.so against tools/ab/libqasr_prev.so
# (the library at the commit of profiles/r5/configs/f16_b64.json), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for v in cur prev; do
    if [ $v = prev ]; then export QASR_LIB_OVERRIDE=$PWD/tools/ab/libqasr_prev.so; else unset QASR_LIB_OVERRIDE; fi
    timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --set-utterances 0 > gpurun_out/ab_$v$i.log 2>&1 || { tail -5 gpurun_out/ab_$v$i.log; exit 1; }
    grep '^{"metric"' gpurun_out/ab_$v$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['stage_ms_per_step_rank0'])"
  done
done
