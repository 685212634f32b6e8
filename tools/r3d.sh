export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libqasr.so libqasr_noslow.so; do
  QASR_LIB_OVERRIDE=$PWD/qwen3-asr.cpp_amd/$lib QASR_FX_DBG=4 QASR_DEV_TRACE=gpurun_out/r3d_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3d_tr.log 2>&1 || exit 1
  echo "== $lib"; python3 tools/trace_report.py gpurun_out/r3d_tr.bin | grep chain
done
