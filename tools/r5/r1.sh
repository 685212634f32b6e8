# round 5 first GPU pass: the whole GPU suite on the cleaned tree (options removed,
# option-coverage tests added), then the single-rounding chain diagnostic
# (var_r1.so: fx8_fast on v_fma_mixlo_f16) against the default, configs[1],
# alternating, and one layer-14 device trace of each (chain cycles per key)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r1_suite.log 2>&1; rc=$?
tail -4 gpurun_out/r1_suite.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r1_suite.log | head -30; exit $rc; }
cp gpurun_out/parity.json gpurun_out/r1_parity.json
for rep in 1 2; do
for L in qwen3-asr.cpp_amd/libqasr.so qwen3-asr.cpp_amd/var_r1.so; do
QASR_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['stage_ms_per_step_rank0']['decode'], [(x['kernel'][:12], x['avg_launch_us']) for x in [d['roofline']]+d['roofline_other']])"
done
done
for L in libqasr var_r1; do
QASR_LIB_OVERRIDE=qwen3-asr.cpp_amd/$L.so QASR_DEV_TRACE=gpurun_out/tr_$L.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/trb.log 2>&1 || { tail -5 gpurun_out/trb.log; exit 1; }
echo "== $L"; python3 tools/trace_report.py gpurun_out/tr_$L.bin 2>&1 | head -8
done
timeout -k 10 400 python -u bench.py > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.log || { tail -5 gpurun_out/r1_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r1_bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('utterance_set')))"
exit 0
