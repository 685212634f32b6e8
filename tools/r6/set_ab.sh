# utterance set A/B on one box: default vs skinny_wdef=1, then a kernel-trace profile of the set (eager)
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in "" "skinny_wdef=1" "" "skinny_wdef=1"; do
  OPT="$o" timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/set_ab.txt 2>&1 || exit 1
done
cd /tmp
QASR_NO_GRAPH=1 N_UTT=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/setprof -o setprof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/r6/set_run.py > $GRAFT_REPO_ROOT/gpurun_out/setprof.log 2>&1 || exit 2
find $GRAFT_REPO_ROOT/gpurun_out/setprof -name "*kernel_trace.csv" -delete
