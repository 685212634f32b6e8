# utterance_set leg (1000 x 30 s) at 64 / 128 / 192 / 256 continuous-batching slots per GPU
export TMPDIR=/tmp
mkdir -p gpurun_out
for S in 64 128 192 256; do
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-slots $S > gpurun_out/slots_$S.json 2> gpurun_out/slots_$S.log || { tail -5 gpurun_out/slots_$S.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/slots_$S.json').read().strip().splitlines()[-1]); u=d['utterance_set']; print($S, u['value'], u['wall_s'], u['rank0_stream'])"
done
exit 0
