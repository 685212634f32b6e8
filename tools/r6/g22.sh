# round-6 GPU job 22: the driver's bench command with 2 and 3 contexts for the utterance set, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for c in 2 3; do
    timeout -k 10 300 python -u bench.py --set-contexts $c > gpurun_out/g22_${c}_${rep}.json 2> gpurun_out/g22.err || { tail gpurun_out/g22.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/g22_${c}_${rep}.json')); u=d['utterance_set']; print('ctx $c', d['value'], u['value'], u['ragged']['value'], u['workload'][-120:-60])" | tee -a gpurun_out/g22.txt
  done
done
