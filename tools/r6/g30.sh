#!/bin/bash
# the gemm8p epilogue's store pattern in isolation
set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/store_pat tools/micro/store_pat.hip > gpurun_out/g30_build.txt 2>&1 &&
timeout -k 10 120 /tmp/store_pat > gpurun_out/g30.txt 2>&1
