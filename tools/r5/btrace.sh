# decode-batch device trace (64 x 30 s, layer 14): the one-launch exact attention's phases
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_DEV_TRACE=gpurun_out/btr.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-utterances 0 > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
python3 tools/r5/batch_trace.py gpurun_out/btr.bin
exit 0
