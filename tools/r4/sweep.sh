# batch-1 delay knobs re-swept on one box (configs[1], 3 timed steps each)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run TAG ENV...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/sw.log 2>&1 || { tail -3 gpurun_out/sw.log; exit 1; }
    grep '^{' gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['stage_ms_per_step_rank0']['decode'])"
}
run base QASR_X=0
run lf QASR_LFFN=1
run lfg10 QASR_LFFN=1 QASR_LFFN_GDELAY=10
run lfg20 QASR_LFFN=1 QASR_LFFN_GDELAY=20
run lfg45 QASR_LFFN=1 QASR_LFFN_GDELAY=45
run lfw25 QASR_LFFN=1 QASR_LFFN_WDELAY=25
run lfw55 QASR_LFFN=1 QASR_LFFN_WDELAY=55
run lfg20w25 QASR_LFFN=1 QASR_LFFN_GDELAY=20 QASR_LFFN_WDELAY=25
exit 0
