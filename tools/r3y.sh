# exact prefill attention variants (PX_KPF: K prefetch, FX_B: chain batch): prefill stage time at 64 x 30 s and configs[1]
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in A B C D A B C D; do
QASR_LIB_OVERRIDE=$PWD/tools/var/libqasr_$n.so timeout -k 10 200 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3y_$n.log 2>&1 || exit 1
QASR_LIB_OVERRIDE=$PWD/tools/var/libqasr_$n.so timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3y1_$n.log 2>&1 || exit 1
a=$(grep '^{' gpurun_out/r3y_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'])")
b=$(grep '^{' gpurun_out/r3y1_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step_rank0'])")
echo "$n | $a | $b"
done
