#!/bin/bash
# does rocprofv3 --pmc work at all here?  control: launch_floor; then the CLI (no python)
source ./gpurun_job.sh
export TMPDIR=/tmp QASR_NO_GRAPH=1
python3 -c "
import sys; sys.path.insert(0,'qwen3-asr.cpp_amd/python'); import qasr
qasr.write_synthetic_gguf('/tmp/full.gguf','full',42,1)
qasr.write_wav('/tmp/c92.wav', qasr.synth_pcm(1000, 92*16000))
"
step pmc_control 60 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_control -o run -- ./tools/launch_floor
step pmc_cli 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemv_kernel -f csv -d gpurun_out/pmc_cli -o run -- ./qwen3-asr.cpp_amd/qwen3-asr-cli -m /tmp/full.gguf -f /tmp/c92.wav --max-tokens 40
