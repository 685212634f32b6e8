export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_$1.log 2>&1; tail -4 gpurun_out/t_$1.log
timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_$1.log 2>&1 || exit 1
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/px_$1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-probe --tok-rate 1 > gpurun_out/px_$1.log 2>&1; echo rc=$?
