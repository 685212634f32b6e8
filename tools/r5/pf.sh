# V^T L2 prefetch distance in the decode chain (fx_decode.h FX_PF): batch trace + utterance set, per library
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in var_pf0 libqasr var_pf3 var_pf4; do
QASR_LIB_OVERRIDE=qwen3-asr.cpp_amd/$L.so QASR_DEV_TRACE=gpurun_out/btr_$L.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 1 --warmup 1 --no-probe --no-cpu-baseline --set-utterances 0 > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
echo "== $L"; python3 tools/r5/batch_trace.py gpurun_out/btr_$L.bin
QASR_LIB_OVERRIDE=qwen3-asr.cpp_amd/$L.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-probe --no-cpu-baseline > gpurun_out/pf.json 2>gpurun_out/pf.log || { tail -5 gpurun_out/pf.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/pf.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['utterance_set']['value'], d['utterance_set']['rank0_stream']['decode_ms'])"
done
exit 0
