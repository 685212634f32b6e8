# round-6 GPU job 25: utterance-set contexts with more hardware queues per process (GPU_MAX_HW_QUEUES=8; the box
# default is 4, which a fourth context plus the default stream exceeded in round 5)
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 3 4; do
  GPU_MAX_HW_QUEUES=8 N_UTT=1000 CTX=$c SLOTS=128 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g25.txt 2>> gpurun_out/g25.err || { tail gpurun_out/g25.err; exit 1; }
  GPU_MAX_HW_QUEUES=8 RAGGED=1 N_UTT=1000 CTX=$c SLOTS=128 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g25.txt 2>> gpurun_out/g25.err || { tail gpurun_out/g25.err; exit 2; }
done
N_UTT=1000 CTX=3 SLOTS=128 REPS=2 timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g25.txt 2>> gpurun_out/g25.err || exit 3
cat gpurun_out/g25.txt
