# fx_vpf 4 (o-proj blocks pull the chain's V^T) against the o-proj weight delay; default (2, 32) beside it
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in "2 32" "4 32" "4 24" "4 40" "6 32" "2 32"; do
set -- $C
QASR_FX_VPF=$1 QASR_FUSE_ODELAY=$2 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/ops_b.log 2>&1 || { tail -5 gpurun_out/ops_b.log; exit 1; }
echo "fx_vpf $1 o_delay $2 $(grep '^{' gpurun_out/ops_b.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
exit 0
