#!/bin/bash
# next-layer QKV in the FFN launch (qkv_ffn): targeted tests, then decode A/B and delay sweep
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 300 --timeout-method thread -k "fused or layer_launch or timeout" > gpurun_out/qf_t.log 2>&1
rc=$?; tail -15 gpurun_out/qf_t.log; [ $rc -ne 0 ] && exit $rc
for cfg in "0 20 10" "1 20 10" "1 10 10" "1 30 10" "1 20 4" "1 20 20"; do
  set -- $cfg
  QASR_QKV_FFN=$1 QASR_QFFN_DELAY=$2 QASR_QFFN_POLL_DELAY=$3 timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/qf_b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/qf_b.log') if l.startswith('{')][-1]); print('qkv_ffn=$1 delay=$2 poll=$3', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'], d['roofline_other'][0]['avg_launch_us'])"
done
