# decode-batch knobs re-swept (f16, 64 x 30 s, 2 timed steps each)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
    local tag=$1; shift
    env "$@" timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/swb.log 2>&1 || { tail -3 gpurun_out/swb.log; exit 1; }
    grep '^{' gpurun_out/swb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['stage_ms_per_step_rank0'])"
}
run base QASR_X=0
run kvnt0 QASR_KV_NT=0
run spl128 QASR_ATT_SPL=128
run stream0 QASR_ATT_STREAM=0
run inf0 QASR_SKINNY_INF=0
run base2 QASR_X=0
exit 0
