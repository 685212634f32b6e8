# round-6 GPU job 9: asymmetric contexts at small shares (the small context starts decoding while the large one prefills)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { N_UTT=$1 CTX=$2 SLOTS=$3 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g9.txt 2>&1; }
run 125 1 125 && run 125 2 32,93 && run 125 2 24,101 && run 125 2 48,77 && run 125 3 16,40,69 && run 250 2 125 && run 250 2 64,128 && run 250 3 32,90,128 || exit 1
