# fx_pipe = 2 with slow groups (default) vs the no-record-path diagnostic library: bench + trace
export TMPDIR=/tmp
mkdir -p gpurun_out

for var in hotv; do
  export QASR_LIB_OVERRIDE=$PWD/tools/var_$var.so
  QASR_FX_PIPE=2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p5_b$var.log 2>&1 || { tail -5 gpurun_out/p5_b$var.log; exit 1; }
  grep '^{' gpurun_out/p5_b$var.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$var', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']])"
  QASR_FX_PIPE=2 QASR_DEV_TRACE=gpurun_out/p5_tr$var.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/p5_trb$var.log 2>&1 || { tail -5 gpurun_out/p5_trb$var.log; exit 1; }
  python3 tools/trace_report.py gpurun_out/p5_tr$var.bin 2>&1 | head -5
done
