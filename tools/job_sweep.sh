#!/bin/bash
# batch-1 fused-launch delays with the fused FFN in place: o-proj weight delay, attention K/V delay
source ./gpurun_job.sh
export TMPDIR=/tmp
step base 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
for o in 12 16 24 28; do QASR_FUSE_ODELAY=$o step od$o 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2; done
for a in 6 14; do QASR_FUSE_DELAY=$a step ad$a 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2; done
for w in 13 15; do QASR_FFN_WDELAY=$w step fw$w 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2; done
step base2 300 ./qwen3-asr.cpp_amd/qasr-bench --steps 5 --warmup 2
