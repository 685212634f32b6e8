# round-6 GPU job 7: torch / RCCL initialised before libqasr.so (bench.py's N > 1 order), 2 and 3 contexts
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 2 3; do
  RCCL=1 CTX=$c timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g7.txt 2>&1 || exit 1
done
for c in 2 3; do
  CTX=$c timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g7.txt 2>&1 || exit 2
done
