# kernel times of the configs[4] aligner leg (transcribe + align, 1 x 92 s)
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/al_prof -o run -- python3 bench.py --pipeline align --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 0.2 > gpurun_out/al_prof.log 2>&1 || { tail -5 gpurun_out/al_prof.log; exit 1; }
head -25 gpurun_out/al_prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
exit 0
