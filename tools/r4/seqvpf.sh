# decode-batch exact attention with the V^T pull (seq_vpf): parity, B=64 bench on/off, conv1 warm timing f16 / q8
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 600 --timeout-method thread -k "fx_seq or configs3 or batch64" > gpurun_out/sv_t.log 2>&1; rc=$?
tail -3 gpurun_out/sv_t.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/sv_t.log | head -20; exit $rc; }
for v in 1 0; do
QASR_SEQ_VPF=$v timeout -k 10 300 python -u bench.py --batch 64 --seconds 30 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sv_b$v.log 2>&1 || { tail -5 gpurun_out/sv_b$v.log; exit 1; }
grep '^{' gpurun_out/sv_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seq_vpf=$v', d['value'], d['stage_ms_per_step_rank0'], [(x['kernel'][:30], x['avg_launch_us'], x['frac']) for x in [d['roofline']]+d['roofline_other']], d['decode_hbm']['frac'])"
done
for q in "" "--q8"; do
QASR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sv_prof$q -o run -- python3 bench.py $q --batch 64 --seconds 30 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --tok-rate 0.2 > gpurun_out/sv_prof$q.log 2>&1 || { tail -5 gpurun_out/sv_prof$q.log; exit 1; }
python3 - "$q" << 'PY'
import csv, sys, glob
f = glob.glob(f"gpurun_out/sv_prof{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
print(sys.argv[1] or "f16", [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in rows if "conv1" in r["Kernel_Name"]],
      [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in rows if "decode_attn_seq" in r["Kernel_Name"]][:6])
PY
done
exit 0
