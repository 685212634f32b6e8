# batch-1 delay knobs re-swept on one box (configs[1], 3 timed steps each)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run TAG ENV...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/sw.log 2>&1 || { tail -3 gpurun_out/sw.log; exit 1; }
    grep '^{' gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['stage_ms_per_step_rank0']['decode'])"
}
run newdefault QASR_X=0
run old QASR_FFN_WDELAY=14 QASR_FUSE_ODELAY=26 QASR_ATT_SPL1=128
run newdefault2 QASR_X=0
exit 0
