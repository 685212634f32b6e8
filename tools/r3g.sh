# stream tests + fused chain perf + configs[3]/[4] drivers
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_api.py -x -v --timeout 280 --timeout-method thread > gpurun_out/r3g_t1.log 2>&1; rc=$?; tail -25 gpurun_out/r3g_t1.log; [ $rc -ne 0 ] && exit $rc
bash tools/r3f.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -x -v -s --timeout 580 --timeout-method thread -k "configs3" > gpurun_out/r3g_t2.log 2>&1; rc=$?; tail -6 gpurun_out/r3g_t2.log; exit $rc
