# round-6 GPU job 24: three set contexts beside an RCCL process group in one process (the N > 1 order: torch +
# RCCL first, then libqasr), then the round's evidence again with the final code (tools/profile_round.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
RCCL=1 N_UTT=1000 CTX=3 SLOTS=128 REPS=2 timeout -k 10 240 python -u tools/r6/set_run.py > gpurun_out/g24_rccl3.txt 2>&1 || { tail -20 gpurun_out/g24_rccl3.txt; exit 1; }
cat gpurun_out/g24_rccl3.txt | grep "^set"
PROF_OUT=gpurun_out/r6prof PROF_CONFIGS=0 bash tools/profile_round.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*agent_info.csv" -delete
