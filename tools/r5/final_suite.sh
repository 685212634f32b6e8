# round-5 evidence: the whole GPU suite (tests/conftest.py records parity.json) + smoke
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread > gpurun_out/r5_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r5_suite.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5_suite.log | head -30; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 || { tail -5 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
exit 0
