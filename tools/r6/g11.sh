# round-6 GPU job 11: the driver's bench command with the configs[1] context closed before the set leg
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/g11_bench.json 2> gpurun_out/g11_bench.err || exit 1
timeout -k 10 300 python -u bench.py --set-contexts 2 > gpurun_out/g11_bench2.json 2> gpurun_out/g11_bench2.err || exit 2
