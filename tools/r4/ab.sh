# A/B: default library vs variants given as arguments (configs[1], 3 timed steps each, alternating)
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for L in qwen3-asr.cpp_amd/libqasr.so "$@"; do
QASR_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['stage_ms_per_step_rank0']['decode'], [(x['kernel'][:12], x['avg_launch_us']) for x in [d['roofline']]+d['roofline_other']])"
done
done
exit 0
