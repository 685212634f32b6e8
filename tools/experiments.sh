#!/bin/bash
# tools/experiments.sh <name> -- the round-2 measurement jobs that DESIGN.md and the
# option comments in csrc/ cite (each ran on a 1-GPU MI355X box through gpurun:
#   gpurun --timeout 900 -- "bash tools/experiments.sh <name>").  Every GPU step
# has its own time limit and a failing step ends the job (no retries).  Names:
#   b64prof    kernel-time breakdown of the batched configs (f16 and Q8_0, 64 x 30 s), decode eager
#   dxq        exact decode chain with 128-key V buffers: Q8_0 tests, configs[1] full test (both decode modes), configs[2] line
#   fxpair     exact decode chain: two query heads per workgroup (shared V^T reads) vs one
#   kvnt       K/V cache loads nontemporal (kv_nt) vs default policy: configs[1] and f16 64 x 30 s
#   lmh        decode-batch LM head tilings (TEMP knob QASR_LMH): kernel time from rocprofv3 stats
#   postnorm   decode batches: RMS norms fused into the o / down projections (post_norm) vs separate launches
#   q8h        Q8_0 prefill / encoder GEMMs on fp16-valued quants (bit-identical): tests + configs[2] line
#   q8ks       Q8_0 tiled GEMM K-stage depth (prefill / encoder of configs[2]) + post_norm bit-identity test
#   q8pmc      what bounds gemm_q8_kernel (configs[2] prefill / encoder): SQ instruction / wait counters, MFMA busy
#   q8t        Q8_0 tiled GEMM tile shapes (TEMP knob QASR_Q8T) on configs[2]
#   qffn       next-layer QKV in the FFN launch (qkv_ffn): targeted tests, then decode A/B and delay sweep
#   qffn2      attention launch without its QKV role: device traces and 64-key splits
#   stream     streamed batch attention splits (att_stream) vs one workgroup per split
#   seq3       per-sequence batch attention with three K/V register sets: tests + 64 x 30 s lines
#   conv1lds   conv1 with the GELU table in LDS: encoder tests + encode times (configs[1], 64 x 30 s)
#   delays     batch-1 fused-launch delays (qkv_delay, o_delay, ffn_wdelay) re-swept on configs[1]
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
case "${1:-}" in
b64prof)
export QASR_NO_GRAPH=1
for q in "" "--q8"; do
  n=b64${q:+_q8}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$n -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline --no-probe $q > gpurun_out/$n.log 2>&1 || { echo "fail $n"; exit 1; }
  python3 - gpurun_out/$n/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:100]}")
PY
done
;;
dxq)
timeout -k 10 400 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dxq_t.log 2>&1
rc=$?; tail -2 gpurun_out/dxq_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "configs1 or configs2" > gpurun_out/dxq_t2.log 2>&1
rc=$?; tail -2 gpurun_out/dxq_t2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dxq_b.log 2>&1 || exit 1
grep "^{" gpurun_out/dxq_b.log > gpurun_out/dxq_c2.json
python3 -c "import json; d=json.load(open('gpurun_out/dxq_c2.json')); print('q8 b64', d['value'], d['stage_ms_per_step_rank0'])"
;;
fxpair)
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
;;
kvnt)
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
;;
lmh)
export QASR_NO_GRAPH=1
for v in 0 1 2 3 4; do
  QASR_LMH=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/lmh$v -o run -- python3 bench.py --batch 64 --seconds 30 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > gpurun_out/lmh$v.log 2>&1 || { echo fail $v; exit 1; }
  python3 - gpurun_out/lmh$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'gemm_skinny_kernel' in r['Name'] and ', 3,' in r['Name'].replace(' ', ' '):
        print(sys.argv[2], r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3)
PY
done
;;
postnorm)
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_q8.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pn_t.log 2>&1
rc=$?; tail -3 gpurun_out/pn_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "batch or configs2" > gpurun_out/pn_t2.log 2>&1
rc=$?; tail -3 gpurun_out/pn_t2.log; [ $rc -ne 0 ] && exit $rc
for pn in 1 0; do
  for q in "" "--q8"; do
    QASR_POST_NORM=$pn timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe $q > gpurun_out/pn_b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pn_b.log') if l.startswith('{')][-1]); print('post_norm=$pn $q', d['value'], d['stage_ms_per_step_rank0']['decode'])"
  done
done
;;
q8h)
timeout -k 10 400 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_batch.py tests/test_gpu_aligner.py -x -q --timeout 300 --timeout-method thread > gpurun_out/q8h_t.log 2>&1
rc=$?; tail -3 gpurun_out/q8h_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread -k "configs2" > gpurun_out/q8h_t2.log 2>&1
rc=$?; tail -3 gpurun_out/q8h_t2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/q8h_b.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/q8h_b.log') if l.startswith('{')][-1]); print('q8 b64', d['value'], d['stage_ms_per_step_rank0'])"
;;
q8ks)
timeout -k 10 400 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ks_t.log 2>&1
rc=$?; tail -3 gpurun_out/ks_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/ks_b.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ks_b.log') if l.startswith('{')][-1]); print('q8 b64', d['value'], d['stage_ms_per_step_rank0'])"
;;
q8pmc)
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
;;
q8t)
for t in 0 1 2; do
  QASR_Q8T=$t timeout -k 10 200 python bench.py --q8 --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/q8t.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/q8t.log') if l.startswith('{')][-1]); print('q8t=$t', d['value'], d['stage_ms_per_step_rank0'])"
done
;;
qffn)
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 300 --timeout-method thread -k "fused or layer_launch or timeout" > gpurun_out/qf_t.log 2>&1
rc=$?; tail -15 gpurun_out/qf_t.log; [ $rc -ne 0 ] && exit $rc
for cfg in "0 20 10" "1 20 10" "1 10 10" "1 30 10" "1 20 4" "1 20 20"; do
  set -- $cfg
  QASR_QKV_FFN=$1 QASR_QFFN_DELAY=$2 QASR_QFFN_POLL_DELAY=$3 timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/qf_b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/qf_b.log') if l.startswith('{')][-1]); print('qkv_ffn=$1 delay=$2 poll=$3', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'], d['roofline_other'][0]['avg_launch_us'])"
done
;;
qffn2)
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
;;
stream)
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_q8.py -x -q --timeout 240 --timeout-method thread > gpurun_out/st_t.log 2>&1
rc=$?; tail -3 gpurun_out/st_t.log; [ $rc -ne 0 ] && exit $rc
for st in 1 0; do
  for q in "" "--q8"; do
    QASR_ATT_STREAM=$st timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline $q > gpurun_out/st_b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/st_b.log') if l.startswith('{')][-1]); print('stream=$st $q', d['value'], d['stage_ms_per_step_rank0']['decode'], d['roofline']['avg_launch_us'])"
  done
done
;;
seq3)
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s3_t.log 2>&1
rc=$?; tail -2 gpurun_out/s3_t.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for q in "" "--q8"; do
    timeout -k 10 200 python bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline --no-probe $q > gpurun_out/s3_b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/s3_b.log') if l.startswith('{')][-1]); print('seq3 $q', d['value'], d['stage_ms_per_step_rank0']['decode'])"
  done
done
;;
conv1lds)
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_q8.py tests/test_hf_anchor.py tests/test_gpu_aligner.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c1_t.log 2>&1
rc=$?; tail -2 gpurun_out/c1_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "encode or configs1" > gpurun_out/c1_t2.log 2>&1
rc=$?; tail -2 gpurun_out/c1_t2.log; [ $rc -ne 0 ] && exit $rc
for a in "" "--batch 64 --seconds 30"; do
  timeout -k 10 200 python bench.py $a --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/c1_b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c1_b.log') if l.startswith('{')][-1]); print('conv1lds $a', d['value'], d['stage_ms_per_step_rank0'])"
done
;;
delays)
for cfg in "10 20 14" "6 20 14" "14 20 14" "10 14 14" "10 26 14" "10 20 10" "10 20 18" "10 20 14" \
           "10 24 14" "10 28 14" "10 32 14" "10 36 14" "6 26 14" "6 28 14" "10 26 14"; do
  set -- $cfg
  QASR_FUSE_DELAY=$1 QASR_FUSE_ODELAY=$2 QASR_FFN_WDELAY=$3 timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/dl_b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dl_b.log') if l.startswith('{')][-1]); print('qkv_delay=$1 o_delay=$2 ffn_wdelay=$3', d['value'], d['stage_ms_per_step_rank0']['decode'])"
done
;;
*)
sed -n 2,23p "$0"; exit 2
;;
esac
