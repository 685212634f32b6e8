# FX_SDEF=1 (the S recurrence inside the chain loop) vs default: bit-identity, layer-14 trace, configs[1] A/B
export TMPDIR=/tmp
# (FX_SDEF: the compile-time variant described in DESIGN.md, removed after this measurement; var_sdef.so is not built any more)
mkdir -p gpurun_out
V=qwen3-asr.cpp_amd/var_sdef.so
QASR_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_full.py -k "fused_launches_match_separate or configs1" > gpurun_out/sd_t.log 2>&1 || { tail -30 gpurun_out/sd_t.log; exit 1; }
tail -1 gpurun_out/sd_t.log
for L in $V qwen3-asr.cpp_amd/libqasr.so; do
QASR_LIB_OVERRIDE=$L QASR_DEV_TRACE=gpurun_out/sd_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/sd_trb.log 2>&1 || { tail -5 gpurun_out/sd_trb.log; exit 1; }
echo $L; python3 tools/trace_report.py gpurun_out/sd_tr.bin 2>&1 | grep -E "chain" | cut -c1-200
done
for L in $V qwen3-asr.cpp_amd/libqasr.so $V qwen3-asr.cpp_amd/libqasr.so; do
QASR_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/sd_b.log 2>&1 || { tail -5 gpurun_out/sd_b.log; exit 1; }
echo "$L $(grep '^{' gpurun_out/sd_b.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
exit 0
