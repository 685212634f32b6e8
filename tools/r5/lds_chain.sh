# decode-batch chain with LDS weights: bit identity (fx_seq one launch vs separate kernels, stream tests) + utterance set
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_batch.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fx_seq or stream or batch or option or configs3" > gpurun_out/ldsc_t.log 2>&1; rc=$?
tail -2 gpurun_out/ldsc_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/ldsc_t.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-contexts 1 > gpurun_out/ldsc_b1.json 2> gpurun_out/ldsc_b1.log || { tail -5 gpurun_out/ldsc_b1.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-probe --no-cpu-baseline > gpurun_out/ldsc_b2.json 2> gpurun_out/ldsc_b2.log || { tail -5 gpurun_out/ldsc_b2.log; exit 1; }
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-probe --no-cpu-baseline --set-utterances 0 > gpurun_out/ldsc_64.json 2> gpurun_out/ldsc_64.log || { tail -5 gpurun_out/ldsc_64.log; exit 1; }
python3 -c "
import json
for f in ['ldsc_b1','ldsc_b2']:
    d=json.loads(open('gpurun_out/%s.json'%f).read().strip().splitlines()[-1]); u=d['utterance_set']
    print(f, u['value'], [(x['prefill_ms'], x['decode_ms']) for x in u['rank0_stream']])
d=json.loads(open('gpurun_out/ldsc_64.json').read().strip().splitlines()[-1]); print('b64', d['value'], d['stage_ms_per_step_rank0'], d['decode_hbm']['frac'])"
