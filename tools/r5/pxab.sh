# prefill exact attention occupancy A/B (64 x 30 s, f16): prefill stage ms per library variant
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base w5b8 w6b4 w6b8 base; do
  L=""; [ $v != base ] && L=qwen3-asr.cpp_amd/var_$v.so
  QASR_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --set-utterances 0 > gpurun_out/pxab_$v.json 2> gpurun_out/pxab_$v.log || { tail -3 gpurun_out/pxab_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/pxab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['stage_ms_per_step_rank0'])"
done
