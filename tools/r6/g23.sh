# round-6 GPU job 23: the down projection at 65..128 rows with every chunk in registers (skinny_bench 128: sums and
# time), the full GPU suite, the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ./tools/skinny_bench 128 > gpurun_out/g23_skinny.txt 2>&1 || { cat gpurun_out/g23_skinny.txt; exit 1; }
cat gpurun_out/g23_skinny.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g23_t.log 2>&1 || { tail -40 gpurun_out/g23_t.log; exit 2; }
tail -2 gpurun_out/g23_t.log
timeout -k 10 300 python -u bench.py > gpurun_out/g23_bench.json 2> gpurun_out/g23_bench.err || { tail gpurun_out/g23_bench.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/g23_bench.json')); u=d['utterance_set']; print(d['value'], d['stage_ms_per_step_rank0'], u['value'], u['ragged']['value'], [ (c['prefill_ms'], c['decode_ms']) for c in u['rank0_stream']])"
