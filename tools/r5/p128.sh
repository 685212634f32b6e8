# kernel stats of a decode-batch run at 64 and 128 clips (eager decode for the profiler)
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for B in 64 128; do
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/p$B -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $B --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --set-utterances 0 > $GRAFT_REPO_ROOT/gpurun_out/p$B.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/p$B.log; exit 1; }
done
exit 0
