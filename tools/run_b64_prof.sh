export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/f16b64_eh.log 2>&1 || exit 1
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/px_b64 -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline --no-probe --tok-rate 0.5 > gpurun_out/px_b64.log 2>&1; echo rc=$?
