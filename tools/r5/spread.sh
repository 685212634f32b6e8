# run-to-run spread of the default bench line on one box: three back-to-back runs
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 600 python -u bench.py > gpurun_out/spread_$i.log 2>&1 || { tail -5 gpurun_out/spread_$i.log; exit 1; }
  grep '^{"metric"' gpurun_out/spread_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); u=d['utterance_set']
print('run $i', d['value'], d['ms_per_step'], d['roofline']['frac'], 'set', u['value'], u['wall_s'])"
done
