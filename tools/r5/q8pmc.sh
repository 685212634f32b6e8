# Q8_0 GEMM counters (tools/micro/q8_gemm_bench): where the register-staged tile's cycles go
export TMPDIR=/tmp
mkdir -p gpurun_out/q8pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/q8pmc -o q8 -- ./tools/micro/q8_gemm_bench > gpurun_out/q8pmc/run.log 2>&1 || { tail -5 gpurun_out/q8pmc/run.log; exit 1; }
find gpurun_out/q8pmc -name "*counter_collection*.csv" | head -3
