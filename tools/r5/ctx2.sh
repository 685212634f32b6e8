# concurrent contexts: the stream test, then the default bench line (utterance_set with 2 contexts)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ctx2_t.log 2>&1; rc=$?
tail -2 gpurun_out/ctx2_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/ctx2_t.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-probe --no-cpu-baseline > gpurun_out/ctx2_b.json 2> gpurun_out/ctx2_b.log || { tail -5 gpurun_out/ctx2_b.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/ctx2_b.json').read().strip().splitlines()[-1]); u=d['utterance_set']
print('headline', d['value']); print('set', u['value'], u['rank0_stream'], u.get('encoder_roofline'))"
