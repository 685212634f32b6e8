# batch-1 delay knobs re-swept on one box (configs[1], 3 timed steps each)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run TAG ENV...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/sw.log 2>&1 || { tail -3 gpurun_out/sw.log; exit 1; }
    grep '^{' gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['stage_ms_per_step_rank0']['decode'])"
}
run base QASR_X=0
run q6 QASR_FUSE_DELAY=6
run q8 QASR_FUSE_DELAY=8
run q12 QASR_FUSE_DELAY=12
run vpf0 QASR_FX_VPF=0
run vpf1 QASR_FX_VPF=1
run vpf3 QASR_FX_VPF=3
run d2 QASR_FFN_DELAY=2
run d6 QASR_FFN_DELAY=6
run o28 QASR_FUSE_ODELAY=28
run o36 QASR_FUSE_ODELAY=36
run base2 QASR_X=0
exit 0
