# PMC passes over the exact prefill attention kernels (tools/micro/px_bench, batch 128 x 405 only)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/px_pmc
mkdir -p $O
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY -d $O/p1 -o p1 --output-format csv -- $GRAFT_REPO_ROOT/tools/micro/px_bench 1 0 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE -d $O/p2 -o p2 --output-format csv -- $GRAFT_REPO_ROOT/tools/micro/px_bench 1 0 || exit 2
find $O -name "*counter_collection.csv" | head
