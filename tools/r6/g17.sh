# round-6 GPU job 17: decode-batch LM head in one launch at 65..128 rows -- bits (lmh128_bench), the full GPU suite,
# the driver's bench command, then one rank's share of the utterance set at N = 8 / 4 / 1 (125 / 250 / 1000 utterances)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/lmh128_bench > gpurun_out/g17_lmh.txt 2>&1 || { cat gpurun_out/g17_lmh.txt; exit 1; }
cat gpurun_out/g17_lmh.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g17_t.log 2>&1 || { tail -40 gpurun_out/g17_t.log; exit 2; }
tail -2 gpurun_out/g17_t.log
timeout -k 10 300 python -u bench.py > gpurun_out/g17_bench.json 2> gpurun_out/g17_bench.err || { tail gpurun_out/g17_bench.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/g17_bench.json')); u=d['utterance_set']; print(d['value'], d['stage_ms_per_step_rank0'], u['value'], u['ragged']['value'], [ (c['prefill_ms'], c['decode_ms']) for c in u['rank0_stream']])"
for spec in "125 1 125" "250 2 125" "1000 2 128"; do
  set -- $spec
  N_UTT=$1 CTX=$2 SLOTS=$3 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g17_share.txt 2>> gpurun_out/g17_share.err || { tail gpurun_out/g17_share.err; exit 4; }
done
cat gpurun_out/g17_share.txt
for st in 60 100 140; do
  N_UTT=125 CTX=2 SLOTS=63 STAGGER_MS=$st REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g17_stagger.txt 2>> gpurun_out/g17_share.err || { tail gpurun_out/g17_share.err; exit 5; }
done
cat gpurun_out/g17_stagger.txt
