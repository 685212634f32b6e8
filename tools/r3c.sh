# fused exact attention: V^T prefetch variants (fx_vpf 0..3), bench + layer-14 trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "match_separate or position_zero" > gpurun_out/r3c_t.log 2>&1; rc=$?; tail -2 gpurun_out/r3c_t.log; [ $rc -ne 0 ] && exit $rc
for v in 2 3 1 0; do
  QASR_FX_VPF=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3c_b$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/r3c_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vpf=$v', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'], d['decode_attention'][-40:])"
done
QASR_DEV_TRACE=gpurun_out/r3c_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3c_tr.log 2>&1 || exit 1
python3 tools/trace_report.py gpurun_out/r3c_tr.bin
