# the 8-phase GEMM in the engine: GEMM bit identity + parity subset, then the utterance set and the default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lds_dma or encode or prefill or stream or option or batch or decode" > gpurun_out/g8e_t.log 2>&1; rc=$?
tail -3 gpurun_out/g8e_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/g8e_t.log | head -30; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-probe --no-cpu-baseline > gpurun_out/g8e_b.json 2> gpurun_out/g8e_b.log || { tail -5 gpurun_out/g8e_b.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/g8e_b.json').read().strip().splitlines()[-1]); u=d['utterance_set']
print('headline', d['value'], d.get('stages_ms')); print('set', u['value'], u['rank0_stream'], u.get('encoder_roofline'))"
exit 0
