# qkv_post 4 heads a wave + o-proj weight pulls under the chain (wpf): parity, benches, trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_aligner.py -x -q --timeout 600 --timeout-method thread -k "prefill or configs3 or batch64 or classes or chunk or fused or configs1" > gpurun_out/wp_t.log 2>&1; rc=$?
tail -3 gpurun_out/wp_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/wp_t.log | head -20; exit $rc; }
for v in 1 0; do
QASR_WPF=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/wp_b$v.log 2>&1 || { tail -5 gpurun_out/wp_b$v.log; exit 1; }
grep '^{' gpurun_out/wp_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wpf=$v', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
done
QASR_DEV_TRACE=gpurun_out/wp_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/wp_trb.log 2>&1 || { tail -5 gpurun_out/wp_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/wp_tr.bin 2>&1 | head -12
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wp_b64.log 2>&1 || { tail -5 gpurun_out/wp_b64.log; exit 1; }
grep '^{' gpurun_out/wp_b64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b64', d['value'], d['stage_ms_per_step_rank0'])"
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/wp_prof -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 0.1 > gpurun_out/wp_prof.log 2>&1 || { tail -5 gpurun_out/wp_prof.log; exit 1; }
grep -h "qkv_post\|prefill_attn" gpurun_out/wp_prof/run_kernel_stats.csv | cut -c1-160
exit 0
