# round-6 GPU job 26: the driver's bench command with 8 hardware queues and four set contexts, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/g26_$rep.json 2> gpurun_out/g26.err || { tail gpurun_out/g26.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g26_$rep.json')); u=d['utterance_set']; print(d['value'], d['stage_ms_per_step_rank0'], u['value'], u['ragged']['value'], u['workload'][150:260], u['roofline']['frac'], u['encoder_roofline']['frac'])" | tee -a gpurun_out/g26.txt
done
