# conv1 at 64 x 30 s: the engine kernel vs the round-4 form, bits + time (tools/micro/conv1_bench.hip)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/conv1_bench > gpurun_out/conv1.txt 2>&1; rc=$?; cat gpurun_out/conv1.txt; exit $rc
