set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/px_bench 5 > gpurun_out/px1.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_aligner.py "tests/test_gpu_full.py::test_full_encoder_poisoned_scratch" "tests/test_gpu_full.py::test_full_prefill_and_steps" "tests/test_gpu_full.py::test_full_encoder_ragged_tiles_bit_identical" > gpurun_out/r6_t1.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r6_b0.json 2> gpurun_out/r6_b0.err || exit 3
