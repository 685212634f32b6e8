# batch-1 fused layer A/B: chain priority, FFN roles in the QKV launch (delays)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <tag> <env...>
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3l_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r3l_$tag.log; exit 1; }
    grep '^{' gpurun_out/r3l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['stage_ms_per_step_rank0']['decode'])"
}
run base QASR_FFN_IN=0
run prio3 QASR_FFN_IN=0 QASR_FX_PRIO=3
run prio1 QASR_FFN_IN=0 QASR_FX_PRIO=1
run in_g0 QASR_FFN_IN=1
run in_g30 QASR_FFN_IN=1 QASR_FFNIN_GWDELAY=30 QASR_FFNIN_WDELAY=30
run in_g30_p3 QASR_FFN_IN=1 QASR_FFNIN_GWDELAY=30 QASR_FFNIN_WDELAY=30 QASR_FX_PRIO=3
run in_g50_d60_p3 QASR_FFN_IN=1 QASR_FFNIN_GWDELAY=50 QASR_FFNIN_WDELAY=50 QASR_FFNIN_DELAY=60 QASR_FX_PRIO=3
for v in "0 0 0 20" "1 30 3 60"; do set -- $v
QASR_FFN_IN=$1 QASR_FFNIN_GWDELAY=$2 QASR_FFNIN_WDELAY=$2 QASR_FX_PRIO=$3 QASR_FFNIN_DELAY=$4 QASR_DEV_TRACE=gpurun_out/r3l_tr$1.bin QASR_DEV_TRACE_LAYER=14 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3l_tr$1.log 2>&1 || exit 1
echo "trace $v"; python3 tools/trace_report.py gpurun_out/r3l_tr$1.bin
done
