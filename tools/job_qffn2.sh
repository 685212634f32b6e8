#!/bin/bash
# attention launch without its QKV role: device traces and 64-key splits
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "0 0" "1 0" "1 64" "0 64"; do
  set -- $cfg
  QASR_QKV_FFN=$1 QASR_ATT_SPL1=$2 QASR_QFFN_DELAY=30 timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/qf_b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/qf_b.log') if l.startswith('{')][-1]); print('qkv_ffn=$1 spl1=$2', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'], d['roofline_other'][0]['avg_launch_us'])"
done
for q in 0 1; do
  QASR_DEV_TRACE=gpurun_out/tr_q$q.bin QASR_DEV_TRACE_LAYER=14 QASR_QKV_FFN=$q QASR_QFFN_DELAY=30 timeout -k 10 150 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-probe > gpurun_out/qf_tr$q.log 2>&1 || exit 1
  python3 tools/trace_report.py gpurun_out/tr_q$q.bin > gpurun_out/tr_q$q.txt 2>&1
  echo "== qkv_ffn=$q"; cat gpurun_out/tr_q$q.txt
done
