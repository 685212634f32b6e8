# the 256x256 8-phase GEMM (csrc/gemm8p.h): element vs LDS-staged wide epilogue, no-store loop, per EPI bit identity
mkdir -p gpurun_out
timeout -k 10 300 ./tools/micro/g8_bench > gpurun_out/g8.txt 2>&1; rc=$?
cat gpurun_out/g8.txt; exit $rc
