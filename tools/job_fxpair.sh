#!/bin/bash
# exact decode chain: two query heads per workgroup (shared V^T reads) vs one
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_batch.py -x -q --timeout 240 --timeout-method thread > gpurun_out/fx_t.log 2>&1
rc=$?; tail -3 gpurun_out/fx_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "configs2 or configs1" > gpurun_out/fx_t2.log 2>&1
rc=$?; tail -3 gpurun_out/fx_t2.log; [ $rc -ne 0 ] && exit $rc
for p in 1; do
  QASR_FX_PAIR=$p timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/fx_b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/fx_b.log') if l.startswith('{')][-1]); print('pair=$p', d['value'], d['stage_ms_per_step_rank0'])"
done
timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/fx_b16.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/fx_b16.log') if l.startswith('{')][-1]); print('f16 b64', d['value'], d['stage_ms_per_step_rank0'])"
timeout -k 10 300 python bench.py --utterances 128 --steps 1 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/fx_utt.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/fx_utt.log') if l.startswith('{')][-1]); print('utt128', d['value'], d.get('stage_ms_per_step_rank0'))"
