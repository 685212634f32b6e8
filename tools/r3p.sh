# decode-batch counters (profiles/r3/batch): f16 and Q8_0, 64 x 30 s
export TMPDIR=/tmp
mkdir -p gpurun_out
PROF_OUT=gpurun_out/prof_batch bash tools/profile_batch.sh || exit 1
for c in f16 q8; do python3 - gpurun_out/prof_batch/$c/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in sorted(d["kernels"], key=lambda k: -k["total_ms"])[:12]:
    print(round(k["total_ms"], 2), k["calls"], k["avg_us"], k["name"][:80], k.get("hbm_read_bytes"), k.get("hbm_write_bytes"), k.get("mfma_util"))
PY
done
