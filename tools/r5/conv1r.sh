# conv1 rows per wave (CONV1_ROWS builds of tools/micro/conv1_bench.hip)
for R in 7; do timeout -k 10 120 ./tools/micro/conv1_bench_r$R || exit 1; done
