# one rank's share of the 1000 x 30 s set at N = 8 / 4 / 2 (125 / 250 / 500 utterances on one GPU)
export TMPDIR=/tmp
mkdir -p gpurun_out
for U in 125 250 500 1000; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-utterances $U > gpurun_out/share_$U.json 2> gpurun_out/share_$U.log || { tail -3 gpurun_out/share_$U.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/share_$U.json').read().strip().splitlines()[-1]); u=d['utterance_set']; print($U, u['value'], u['wall_s'], u['workload'][-120:])"
done
