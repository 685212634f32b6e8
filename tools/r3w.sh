# V^T read-ahead clamped to the sequence's last key block: full GPU suite, 64 x 30 s line, configs[1] line, batch kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 580 --timeout-method thread > gpurun_out/r3w_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3w_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3w_t.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3w_b64.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3w_b1.log 2>&1 || exit 1
for f in gpurun_out/r3w_b64.log gpurun_out/r3w_b1.log; do grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3w_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r3w_prof.log 2>&1 || exit 1
