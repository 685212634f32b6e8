# the default bench line (as the driver runs it) with the round-5 profiles in place
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r5_bench.log 2>&1 || { tail -5 gpurun_out/r5_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/r5_bench.log > gpurun_out/r5_bench.json
python3 -c "
import json; d=json.loads(open('gpurun_out/r5_bench.json').read())
u=d['utterance_set']
print(d['value'], d['roofline']['frac'], d['roofline']['traffic_source'], d['encoder_roofline']['frac'], d['encoder_roofline']['profiled'].get('source'))
print('set', u['value'], u['encoder_roofline'])
print('cpu', d['cpu_baseline']['value'])"
