# Q8_0 GEMM on the LDS-DMA ring: bit identity vs the register-staged tile, Q8 tests,
# Q8_0 64 x 30 s line (encode / prefill ms)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_full.py tests/test_gpu_q8.py -k "q8 or Q8 or configs2" > gpurun_out/q8d_tests.log 2>&1 || { tail -30 gpurun_out/q8d_tests.log; exit 1; }
grep -E "PASS|FAIL|SKIP" gpurun_out/q8d_tests.log | cut -c1-120; tail -2 gpurun_out/q8d_tests.log
timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --set-utterances 0 > gpurun_out/q8d_bench.log 2>&1 || { tail -5 gpurun_out/q8d_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/q8d_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'])"
