# round-3 evidence: full -m gpu suite, smoke, bench + configs lines + rocprofv3 stats / PMC passes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread > gpurun_out/r3o_t.log 2>&1; rc=$?; grep -E "FAIL|ERROR" gpurun_out/r3o_t.log | head; tail -2 gpurun_out/r3o_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3o_s.log 2>&1 || { tail gpurun_out/r3o_s.log; exit 1; }
PROF_OUT=gpurun_out/prof_r3 PROF_CONFIGS=1 bash tools/profile_round.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/prof_r3/bench.json')); print(d['value'], d['stage_ms_per_step_rank0'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['cpu_baseline']['value'])"
