# round-6 GPU job 6: contexts per GPU for the utterance set, with and without a live RCCL process group
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 2 3 2 3; do
  CTX=$c timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g6_ctx.txt 2>&1 || exit 1
done
for c in 2 3; do
  RCCL=1 CTX=$c timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g6_ctx.txt 2>&1 || exit 2
done
N_UTT=125 CTX=1 SLOTS=125 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g6_ctx.txt 2>&1 || exit 3
N_UTT=125 CTX=2 SLOTS=63 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g6_ctx.txt 2>&1 || exit 3
