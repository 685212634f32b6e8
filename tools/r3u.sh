# 8-wave LDS-DMA GEMM tiles + FFN weights pulled into L2 during the chain: tests, A/B lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py tests/test_gpu_aligner.py tests/test_hf_anchor.py -x -q --timeout 580 --timeout-method thread -k "not two_threads and not wait_timeout" > gpurun_out/r3u_t.log 2>&1; rc=$?; tail -3 gpurun_out/r3u_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3u_t.log | head; exit $rc; }
for v in "1 30" "0 30" "1 10" "1 50"; do set -- $v
QASR_FFN_PF=$1 QASR_FFN_PF_DELAY=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3u_b$1_$2.log 2>&1 || exit 1
grep '^{' gpurun_out/r3u_b$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pf $1 $2', d['value'], d['stage_ms_per_step_rank0'], d['encoder_roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r3u_b64.log 2>&1 || exit 1
grep '^{' gpurun_out/r3u_b64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b64', d['value'], d['stage_ms_per_step_rank0'], d['encoder_roofline']['frac'])"
