# fx_pipe 4 device trace: chain rate, barrier waits, loader write times (layer 14)
# (fx_pipe 4 = the loader-ring chain of commit 34c4760, removed after this measurement)
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_FX_PIPE=4 QASR_DEV_TRACE=gpurun_out/ring_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/ring_trb.log 2>&1 || { tail -5 gpurun_out/ring_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/ring_tr.bin 2>&1 | grep -E "chain" | cut -c1-200
python3 tools/r4/ring_probe.py gpurun_out/ring_tr.bin
