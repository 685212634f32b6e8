# Q8_0 GEMM: register-staged tile vs the LDS-DMA ring (tools/micro/q8_gemm_bench.hip)
timeout -k 10 300 ./tools/micro/q8_gemm_bench > gpurun_out/q8g.txt 2>&1; rc=$?; cat gpurun_out/q8g.txt; exit $rc
