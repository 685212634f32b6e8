# V^T for the chain pulled by the o-proj blocks of its XCD (fx_vpf 4) instead of by the chain workgroups (2, default)
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in 4 6 2; do
QASR_FX_VPF=$V QASR_DEV_TRACE=gpurun_out/op_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/op_trb.log 2>&1 || { tail -5 gpurun_out/op_trb.log; exit 1; }
echo "fx_vpf $V"; python3 tools/trace_report.py gpurun_out/op_tr.bin 2>&1 | grep -E "chain" | cut -c1-200
python3 tools/r4/wave_probe.py gpurun_out/op_tr.bin | grep gather | head -2
done
for V in 4 2 4 2; do
QASR_FX_VPF=$V timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/op_b.log 2>&1 || { tail -5 gpurun_out/op_b.log; exit 1; }
echo "fx_vpf $V $(grep '^{' gpurun_out/op_b.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
exit 0
