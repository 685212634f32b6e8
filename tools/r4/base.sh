# round-4 baseline: default bench line (no CPU baseline) on a fresh box
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r4_base.log 2>&1 || { tail -5 gpurun_out/r4_base.log; exit 1; }
grep '^{' gpurun_out/r4_base.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
