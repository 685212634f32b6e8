# decode-batch device trace (128 x 30 s, layer 14): the one-launch exact attention's phases
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_DEV_TRACE=gpurun_out/btr128.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 300 python -u bench.py --batch 128 --seconds 30 --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-utterances 0 > gpurun_out/btr128.log 2>&1 || { tail -5 gpurun_out/btr128.log; exit 1; }
python3 tools/r5/batch_trace.py gpurun_out/btr128.bin
exit 0
