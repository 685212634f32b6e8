# round-6 GPU job 15: the round-6 exact prefill kernel in the product -- px_bench bits, the full GPU suite, the bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 ./tools/micro/px_bench 4 > gpurun_out/g15_px.txt 2>&1 || { cat gpurun_out/g15_px.txt; exit 1; }
cat gpurun_out/g15_px.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g15_t.log 2>&1 || { tail -40 gpurun_out/g15_t.log; exit 2; }
tail -3 gpurun_out/g15_t.log
timeout -k 10 300 python -u bench.py > gpurun_out/g15_bench.json 2> gpurun_out/g15_bench.err || { tail gpurun_out/g15_bench.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/g15_bench.json')); u=d['utterance_set']; print(d['value'], d['stage_ms_per_step_rank0'], u['value'], u['ragged']['value'], [ (c['prefill_ms'], c['decode_ms']) for c in u['rank0_stream']])"
