#!/bin/bash
# gemm8p persistent grid / staggered starts A/B on the encoder / prefill shapes
set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o /tmp/g8_bench tools/micro/g8_bench.hip > gpurun_out/g29_build.txt 2>&1 &&
timeout -k 10 400 /tmp/g8_bench > gpurun_out/g29.txt 2>&1
