# Q8_0 block dot with the biased-accumulator int->fp32 conversion: Q8 parity tests
# (bit-identity of every Q8 path vs the oracle bars) and the Q8_0 64 x 30 s line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_q8.py -k "not nothing" > gpurun_out/q8b_tests.log 2>&1 || { tail -20 gpurun_out/q8b_tests.log; exit 1; }
tail -3 gpurun_out/q8b_tests.log
timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --set-utterances 0 > gpurun_out/q8b_bench.log 2>&1 || { tail -5 gpurun_out/q8b_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/q8b_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'])"
