# 256-row LDS-DMA GEMM tiles (8 waves) on the encoder / prefill shapes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/micro/glds_gemm_bench 1 > gpurun_out/r3s_gemm.log 2>&1; rc=$?; cat gpurun_out/r3s_gemm.log; exit $rc
