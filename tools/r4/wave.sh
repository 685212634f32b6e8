# default chain: per-wave chain end and cycles a key (layer 14 device trace)
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_DEV_TRACE=gpurun_out/wv_tr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/wv_trb.log 2>&1 || { tail -5 gpurun_out/wv_trb.log; exit 1; }
python3 tools/trace_report.py gpurun_out/wv_tr.bin 2>&1 | cut -c1-230
python3 tools/r4/wave_probe.py gpurun_out/wv_tr.bin
