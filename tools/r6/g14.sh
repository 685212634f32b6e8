# round-6 GPU job 14: prefill_attn_exact4_kernel (sign-encoded words, per-key scale) against the product kernel,
# every px_bench case bit for bit, then one VALU PMC pass at 128 x 405
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 ./tools/micro/px_bench 6 > gpurun_out/g14_px.txt 2>&1 || { cat gpurun_out/g14_px.txt; exit 1; }
cat gpurun_out/g14_px.txt
O=$GRAFT_REPO_ROOT/gpurun_out/g14_pmc
mkdir -p $O
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY -d $O/p1 -o p1 --output-format csv -- $GRAFT_REPO_ROOT/tools/micro/px_bench 1 0 > $O/p1.log 2>&1 || exit 2
python3 $GRAFT_REPO_ROOT/tools/r6/pmc_sum.py $O/p1 || true
