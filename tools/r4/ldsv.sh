# diagnostic: the chain with V read from LDS (wrong values) -- its cycles a key in place
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in qwen3-asr.cpp_amd/var_ldsv.so qwen3-asr.cpp_amd/libqasr.so; do
QASR_LIB_OVERRIDE=$L QASR_DEV_TRACE=gpurun_out/lv_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/lv_trb.log 2>&1 || { tail -5 gpurun_out/lv_trb.log; exit 1; }
echo $L; python3 tools/trace_report.py gpurun_out/lv_tr.bin 2>&1 | grep -E "chain" | cut -c1-200
done
exit 0
