# Q8_0 GEMM with VGPR-form int8 MFMA results: Q8 parity, configs[2] bench, kernel times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_full.py -x -q --timeout 600 --timeout-method thread -k "q8" > gpurun_out/q8_t.log 2>&1; rc=$?
tail -3 gpurun_out/q8_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/q8_t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/q8_b.log 2>&1 || { tail -5 gpurun_out/q8_b.log; exit 1; }
grep '^{' gpurun_out/q8_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q8 b64', d['value'], d['stage_ms_per_step_rank0'])"
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/q8_prof -o run -- python3 bench.py --q8 --batch 64 --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 0.1 > gpurun_out/q8_prof.log 2>&1 || { tail -5 gpurun_out/q8_prof.log; exit 1; }
grep -h "gemm_q8\|conv1" gpurun_out/q8_prof/run_kernel_stats.csv | cut -c1-150
exit 0
