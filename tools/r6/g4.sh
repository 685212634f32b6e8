# round-6 GPU job 4: the full GPU suite on the new defaults, then the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/g4_t.log 2>&1 || { tail -40 gpurun_out/g4_t.log; exit 1; }
tail -3 gpurun_out/g4_t.log
