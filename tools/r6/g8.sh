# round-6 GPU job 8: contexts x slots at one rank's share of the set (N = 8 / 4 / 2 on one GPU)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { N_UTT=$1 CTX=$2 SLOTS=$3 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g8.txt 2>&1; }
run 125 1 125 && run 125 2 63 && run 125 3 42 && run 250 2 125 && run 250 3 84 && run 500 2 128 && run 500 3 128 || exit 1
