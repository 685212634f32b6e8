# round-6 GPU job 5: exact prefill attention (branch-free weights) A/B, the full GPU suite, the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 ./tools/micro/px_bench 6 > gpurun_out/g5_px.txt 2>&1 || exit 1
cat gpurun_out/g5_px.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g5_t.log 2>&1 || { tail -40 gpurun_out/g5_t.log; exit 2; }
tail -3 gpurun_out/g5_t.log
timeout -k 10 300 python -u bench.py > gpurun_out/g5_bench.json 2> gpurun_out/g5_bench.err || exit 3
