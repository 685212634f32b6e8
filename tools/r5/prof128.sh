# kernel stats of a 128 x 30 s batch (eager decode, QASR_NO_GRAPH=1), one warm-up step; top kernels printed
export TMPDIR=/tmp
D=gpurun_out/prof128; mkdir -p $D
QASR_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $D -o run -- python3 bench.py --batch 128 --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 1.0 --set-utterances 0 > gpurun_out/prof128.log 2>&1 || { tail -5 gpurun_out/prof128.log; exit 1; }
f=$(find $D -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/prof128_stats.csv
python3 - <<'PY'
import csv
r=list(csv.DictReader(open('gpurun_out/prof128_stats.csv')))
tot=sum(float(x['TotalDurationNs']) for x in r)
for x in r[:28]: print(f"{x['Name'][:90]:90s} {x['Calls']:>6} {float(x['TotalDurationNs'])/1e6:9.2f} ms {float(x['AverageNs'])/1e3:9.1f} us")
print('total', tot/1e6, 'ms')
PY
