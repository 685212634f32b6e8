# round-6 GPU job 2: new option tests, set A/B (skinny_wdef, refill_group at share sizes), bench line, set profile
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py "tests/test_gpu_full.py::test_full_option_matches_default" > gpurun_out/g2_t.log 2>&1 || { tail -30 gpurun_out/g2_t.log; exit 1; }
tail -3 gpurun_out/g2_t.log
for o in "" "skinny_wdef=1" "" "skinny_wdef=1"; do
  OPT="$o" timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g2_set.txt 2>&1 || exit 2
done
for g in 0 16 32; do
  N_UTT=125 SLOTS=63 OPT="refill_group=$g" timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g2_share.txt 2>&1 || exit 3
  N_UTT=250 SLOTS=125 OPT="refill_group=$g" timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g2_share.txt 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err || exit 4
cd /tmp
QASR_NO_GRAPH=1 N_UTT=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/setprof -o setprof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/r6/set_run.py > $GRAFT_REPO_ROOT/gpurun_out/setprof.log 2>&1 || exit 5
find $GRAFT_REPO_ROOT/gpurun_out/setprof -name "*kernel_trace.csv" -delete
