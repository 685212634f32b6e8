# round-6 GPU job 10: torch-first engine test, then the driver's bench command (3 contexts by the share policy)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_api.py::test_engine_after_torch_rccl_in_one_process" > gpurun_out/g10_t.log 2>&1 || { tail -30 gpurun_out/g10_t.log; exit 1; }
tail -2 gpurun_out/g10_t.log
timeout -k 10 300 python -u bench.py > gpurun_out/g10_bench.json 2> gpurun_out/g10_bench.err || exit 2
