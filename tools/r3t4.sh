# configs[1] trace: the chain's shader-clock rate (cycles a key, GHz)
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_DEV_TRACE=gpurun_out/r3t4_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3t4_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3t4_tr.bin
