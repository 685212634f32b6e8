# the 65..128-row LM head (two row-half launches): option bit-identity at 100 rows, then the utterance set at 64 / 128 slots
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "lmh" > gpurun_out/lmh.log 2>&1; rc=$?
tail -3 gpurun_out/lmh.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/lmh.log | head; exit $rc; }
for S in 64 128; do
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-slots $S > gpurun_out/s$S.json 2> gpurun_out/s$S.log || { tail -5 gpurun_out/s$S.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s$S.json').read().strip().splitlines()[-1]); u=d['utterance_set']; print($S, u['value'], u['rank0_stream'])"
done
exit 0
