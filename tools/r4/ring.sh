# the loader-ring chain (fx_pipe 4): bit-identity, layer-14 device trace, configs[1] A/B
# (fx_pipe 4 = the loader-ring chain of commit 34c4760, removed after this measurement)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_full.py -k "fused_launches_match_separate and (FX_PIPE4 or FX_PIPE3)" > gpurun_out/ring_t.log 2>&1 || { tail -30 gpurun_out/ring_t.log; exit 1; }
tail -2 gpurun_out/ring_t.log
for P in 0 4; do
QASR_FX_PIPE=$P QASR_DEV_TRACE=gpurun_out/ring_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/ring_trb.log 2>&1 || { tail -5 gpurun_out/ring_trb.log; exit 1; }
echo "fx_pipe $P"; python3 tools/trace_report.py gpurun_out/ring_tr.bin 2>&1 | grep -E "chain|attention" | cut -c1-220
done
for P in 0 4 0 4; do
QASR_FX_PIPE=$P timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/ring_b$P.log 2>&1 || { tail -5 gpurun_out/ring_b$P.log; exit 1; }
echo "fx_pipe $P $(tail -1 gpurun_out/ring_b$P.log | cut -c1-90)"
done
exit 0
