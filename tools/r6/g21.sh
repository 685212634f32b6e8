# round-6 GPU job 21: contexts per GPU again after the round's kernel changes (1000 x 30 s and the ragged set, 2 vs 3 x 128 slots)
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for c in 2 3; do
    N_UTT=1000 CTX=$c SLOTS=128 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g21.txt 2>> gpurun_out/g21.err || { tail gpurun_out/g21.err; exit 1; }
    RAGGED=1 N_UTT=1000 CTX=$c SLOTS=128 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g21.txt 2>> gpurun_out/g21.err || { tail gpurun_out/g21.err; exit 2; }
  done
done
cat gpurun_out/g21.txt
