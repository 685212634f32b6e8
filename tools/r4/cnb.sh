# chain V^T depth variant (var_cnb3.so: FX_CNB=3, o-proj 2 rows a wave) vs default: bench + trace + fused parity
export TMPDIR=/tmp
mkdir -p gpurun_out
V=qwen3-asr.cpp_amd/var_cnb3.so
QASR_LIB_OVERRIDE=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "fused_launches_match or configs1" > gpurun_out/cn_t.log 2>&1; rc=$?
tail -2 gpurun_out/cn_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/cn_t.log | head -20; exit $rc; }
for L in $V qwen3-asr.cpp_amd/libqasr.so; do
QASR_LIB_OVERRIDE=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/cn_b.log 2>&1 || { tail -5 gpurun_out/cn_b.log; exit 1; }
grep '^{' gpurun_out/cn_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['stage_ms_per_step_rank0']['decode'], [(x['kernel'][:20], x['avg_launch_us']) for x in [d['roofline']]+d['roofline_other']])"
done
QASR_LIB_OVERRIDE=$V QASR_DEV_TRACE=gpurun_out/cn_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/cn_trb.log 2>&1 || { tail -5 gpurun_out/cn_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/cn_tr.bin 2>&1 | head -5
exit 0
