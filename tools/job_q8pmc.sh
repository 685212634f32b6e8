#!/bin/bash
# what bounds gemm_q8_kernel (configs[2] prefill / encoder): SQ instruction / wait counters, MFMA busy
export TMPDIR=/tmp
mkdir -p gpurun_out
B="./qwen3-asr.cpp_amd/qasr-bench --q8 --batch 64 --seconds 30 --steps 1 --warmup 0 --tok-rate 0.05"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "gemm_q8_kernel|gemm_glds" -f csv -d gpurun_out/q8pmc1 -o run -- $B > gpurun_out/q8pmc1.log 2>&1 || { echo fail1; tail -5 gpurun_out/q8pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE --kernel-include-regex "gemm_q8_kernel|gemm_glds" -f csv -d gpurun_out/q8pmc2 -o run -- $B > gpurun_out/q8pmc2.log 2>&1 || { echo fail2; tail -5 gpurun_out/q8pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "gemm_q8_kernel|gemm_glds" -f csv -d gpurun_out/q8pmc3 -o run -- $B > gpurun_out/q8pmc3.log 2>&1 || { echo fail3; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in ("q8pmc1", "q8pmc2"):
    for f in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()): print(f"   {c:32s} {x:.4g}")
for f in glob.glob("gpurun_out/q8pmc3/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)): print(r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3)
PY
