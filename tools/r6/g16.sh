# round-6 GPU job 16: the decode-batch LM head at 65..128 rows in one launch (tools/micro/lmh128_bench: bits and time)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/lmh128_bench > gpurun_out/g16_lmh.txt 2>&1; rc=$?
cat gpurun_out/g16_lmh.txt
exit $rc
