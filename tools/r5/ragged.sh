export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ragged or lds_dma" > gpurun_out/ragged.log 2>&1; rc=$?
tail -3 gpurun_out/ragged.log; [ $rc -ne 0 ] && grep -E "Error|assert" gpurun_out/ragged.log | head; exit $rc
