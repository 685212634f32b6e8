# qkv_post 4 heads a wave: prefill parity (tiny + full), B=64 bench, qkv_post timing
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_aligner.py -x -q --timeout 600 --timeout-method thread -k "prefill or configs3 or batch64 or classes or chunk" > gpurun_out/qp_t.log 2>&1; rc=$?
tail -3 gpurun_out/qp_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/qp_t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/qp_b.log 2>&1 || { tail -5 gpurun_out/qp_b.log; exit 1; }
grep '^{' gpurun_out/qp_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b64', d['value'], d['stage_ms_per_step_rank0'])"
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/qp_prof -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 0.1 > gpurun_out/qp_prof.log 2>&1 || { tail -5 gpurun_out/qp_prof.log; exit 1; }
grep -h "qkv_post\|prefill_attn" gpurun_out/qp_prof/run_kernel_stats.csv | cut -c1-200
exit 0
