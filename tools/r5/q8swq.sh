# decode-batch Q8_0 gate/up with the down projection's quantisation in its epilogue:
# bits + tilings (tools/skinny_q8_bench.hip), Q8 tests, Q8_0 64 x 30 s line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/skinny_q8_bench 64 > gpurun_out/skq8_64.txt 2>&1; rc=$?; cat gpurun_out/skq8_64.txt; [ $rc = 0 ] || exit 1
timeout -k 10 120 ./tools/skinny_q8_bench 23 > gpurun_out/skq8_23.txt 2>&1; rc=$?; head -3 gpurun_out/skq8_23.txt; [ $rc = 0 ] || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_q8.py tests/test_gpu_full.py -k "q8 or Q8 or configs2" > gpurun_out/q8s_tests.log 2>&1 || { tail -30 gpurun_out/q8s_tests.log; exit 1; }
grep -E "PASS|FAIL|SKIP" gpurun_out/q8s_tests.log | cut -c1-120; tail -2 gpurun_out/q8s_tests.log
timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --set-utterances 0 > gpurun_out/q8s_bench.log 2>&1 || { tail -5 gpurun_out/q8s_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/q8s_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'])"
