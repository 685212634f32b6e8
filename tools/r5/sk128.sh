# decode-batch GEMM tilings at 128 rows (tools/skinny_bench.hip)
mkdir -p gpurun_out
timeout -k 10 300 ./tools/skinny_bench 128 > gpurun_out/sk128.txt 2>&1; rc=$?
cat gpurun_out/sk128.txt; exit $rc
