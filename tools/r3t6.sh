# chain cycles a key against the V^T pull variants (fx_vpf 0..3)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2 3; do
QASR_FX_VPF=$v QASR_DEV_TRACE=gpurun_out/r3t6_$v.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3t6_$v.log 2>&1 || exit 1
echo "fx_vpf=$v"; python3 tools/trace_report.py gpurun_out/r3t6_$v.bin | grep -E "chain"
grep '^{' gpurun_out/r3t6_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0']['decode'])"
done
