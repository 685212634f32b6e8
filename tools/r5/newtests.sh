# the round-5 API-completeness and stream tests on the GPU
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refapi.py tests/test_gpu_full.py -x -v --timeout 500 --timeout-method thread -k "with_audio_after or no_chunk or stream_34" > gpurun_out/newtests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/newtests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/skinny_bench 64 > gpurun_out/skinny64.txt 2>&1; cat gpurun_out/skinny64.txt
exit 0
