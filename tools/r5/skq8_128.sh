# decode-batch Q8_0 GEMM tilings at 128 rows (tools/skinny_q8_bench.hip)
timeout -k 10 180 ./tools/skinny_q8_bench 128 > gpurun_out/skq8_128.txt 2>&1; rc=$?; cat gpurun_out/skq8_128.txt; exit $rc
