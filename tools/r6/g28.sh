# round-6 GPU job 28: contexts per GPU by share with 8 (16) hardware queues a process
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { GPU_MAX_HW_QUEUES=$1 N_UTT=$2 CTX=$3 SLOTS=128 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py 2>> gpurun_out/g28.err | sed "s/^/hwq $1: /" >> gpurun_out/g28.txt; }
run 8 1000 5 || exit 1
run 16 1000 6 || exit 2
run 16 1000 4 || exit 3
run 8 500 3 || exit 4
run 8 500 4 || exit 5
run 8 250 2 || exit 6
run 8 250 3 || exit 7
run 8 125 1 || exit 8
run 8 125 2 || exit 9
cat gpurun_out/g28.txt
