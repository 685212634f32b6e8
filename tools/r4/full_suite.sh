# the whole GPU suite (records profiles' parity.json through tests/conftest.py) + smoke
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/fs_t.log 2>&1; rc=$?
tail -5 gpurun_out/fs_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/fs_t.log | head -30; exit $rc; }
exit 0
