# round-6 GPU job 27: the full GPU suite (with the expf self-check), then the round's evidence with the final code
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g27_t.log 2>&1 || { tail -40 gpurun_out/g27_t.log; exit 2; }
grep -E "expf|passed|failed" gpurun_out/g27_t.log | tail -3
rm -rf gpurun_out/r6prof
PROF_OUT=gpurun_out/r6prof PROF_CONFIGS=0 bash tools/profile_round.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*agent_info.csv" -delete
