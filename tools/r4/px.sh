# prefill exact attention asm fast path: bit-identity vs the compiler's (var_pxold.so), timings
export TMPDIR=/tmp
mkdir -p gpurun_out
QASR_VARIANT=qwen3-asr.cpp_amd/var_pxold.so timeout -k 10 600 python -u tools/r4/px_check.py || exit 1
for L in qwen3-asr.cpp_amd/libqasr.so qwen3-asr.cpp_amd/var_pxold.so; do
QASR_LIB_OVERRIDE=$L timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/px_b.log 2>&1 || { tail -5 gpurun_out/px_b.log; exit 1; }
grep '^{' gpurun_out/px_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L b64', d['value'], d['stage_ms_per_step_rank0'])"
QASR_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/r4/align_time.py 2>&1 | tail -1
done
exit 0
