export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/r5/two_ctx.py > gpurun_out/two_ctx.txt 2>&1; rc=$?
cat gpurun_out/two_ctx.txt | tail -8; exit $rc
