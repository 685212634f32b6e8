# decode-batch GEMM tilings at 64 rows: the engine's and the 128-row set (tools/skinny_bench.hip)
mkdir -p gpurun_out
timeout -k 10 200 ./tools/skinny_bench 64 > gpurun_out/sk64.txt 2>&1 && SKINNY_ALT=1 timeout -k 10 200 ./tools/skinny_bench 64 > gpurun_out/sk64_alt.txt 2>&1; rc=$?
cat gpurun_out/sk64.txt gpurun_out/sk64_alt.txt | grep -v "^M =\|empty"; exit $rc
