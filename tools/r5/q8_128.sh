# Q8_0 decode batches at 65..128 rows: Q8 tests (incl. the 100-row skinny bit identity) + the
# configs[2] line with its Q8_0 utterance set (128 slots a context)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_q8.py tests/test_gpu_full.py -k "q8 or Q8 or configs2" > gpurun_out/q8r_tests.log 2>&1 || { tail -30 gpurun_out/q8r_tests.log; exit 1; }
tail -1 gpurun_out/q8r_tests.log
timeout -k 10 400 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/q8r_bench.log 2>&1 || { tail -5 gpurun_out/q8r_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/q8r_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], 'set', d['utterance_set']['value'])"
