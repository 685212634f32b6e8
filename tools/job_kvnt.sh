#!/bin/bash
# K/V cache loads nontemporal (kv_nt) vs default policy: configs[1] and f16 64 x 30 s
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/nt_t.log 2>&1
rc=$?; tail -2 gpurun_out/nt_t.log; [ $rc -ne 0 ] && exit $rc
for nt in 0 1 0 1; do
  QASR_KV_NT=$nt timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/nt_b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/nt_b.log') if l.startswith('{')][-1]); print('kv_nt=$nt c1', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'])"
done
for nt in 0 1; do
  QASR_KV_NT=$nt timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/nt_b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/nt_b.log') if l.startswith('{')][-1]); print('kv_nt=$nt b64', d['value'], d['stage_ms_per_step_rank0']['decode'])"
done
