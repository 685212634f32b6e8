# conv1 rework: encoder / conv parity tests, batch encoder bit identities, 64 x 30 s f16 line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_q8.py tests/test_gpu_full.py -k "encode or conv or ragged or lds_dma or batch64 or configs3 or configs1" > gpurun_out/c1_tests.log 2>&1 || { tail -30 gpurun_out/c1_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/c1_tests.log; tail -1 gpurun_out/c1_tests.log
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --set-utterances 0 > gpurun_out/c1_bench.log 2>&1 || { tail -5 gpurun_out/c1_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/c1_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], d['encoder_roofline']['frac'])"
