# decode batches: exact attention (scores + chain) in one launch -- bit-identity, A/B at 64 x 30 s, kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_q8.py -x -v --timeout 580 --timeout-method thread -k "fx_seq or batch or configs3 or stream or configs2 or q8" > gpurun_out/r3x_t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/r3x_t.log | tail -40; tail -3 gpurun_out/r3x_t.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
QASR_FX_SEQ=$v timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3x_b$v.log 2>&1 || exit 1
grep '^{' gpurun_out/r3x_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fx_seq=$v', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3x_q8.log 2>&1 || exit 1
grep '^{' gpurun_out/r3x_q8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q8', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r3x_prof -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline --no-probe --tok-rate 0.5 > gpurun_out/r3x_prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r3x_prof/**/*kernel_stats.csv', recursive=True)[0]
for x in sorted(csv.DictReader(open(f)), key=lambda x: -float(x['TotalDurationNs']))[:14]:
    print(x['Name'][:90], x['Calls'], x['AverageNs'])
PY
