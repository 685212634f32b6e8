"""Per-launch start / end of one decode-batch layer (QKV norm .. down) from a
rocprofv3 kernel trace (tools/profile_batch.sh's stats pass: eager launches,
QASR_NO_GRAPH=1, so the gaps hold host dispatch and are wider than in the
replayed graph; the durations are the kernels').  Picks decoder layer L of the
middle decode step.  Dev tool:  python tools/r5/group_trace.py trace.csv [L]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
layer = int(sys.argv[2]) if len(sys.argv) > 2 else 14
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a decode-batch layer starts at the attention-norm launch that precedes a skinny QKV GEMM
# followed by decode_attn_seq_kernel
name = [r["Kernel_Name"] for r in rows]
starts = [i for i in range(len(rows) - 2)
          if "rmsnorm_kernel" in name[i] and "gemm_skinny" in name[i + 1] and "decode_attn_seq" in name[i + 2]]
if not starts:
    sys.exit("no decode-batch layer found")
# group layer starts into steps (28 consecutive layers; the LM head separates steps)
steps, cur = [], []
for i in starts:
    if cur and any("lmhead" in n for n in name[cur[-1]:i]):
        steps.append(cur)
        cur = []
    cur.append(i)
steps.append(cur)
step = steps[len(steps) // 2]
i0 = step[layer]
i1 = step[layer + 1] if layer + 1 < len(step) else i0 + 7
t0 = int(rows[i0]["Start_Timestamp"])
print(f"decode step {len(steps) // 2} of {len(steps)}, layer {layer}: launch, start / end (us from the layer's first start), duration")
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"  {r['Kernel_Name'][:64]:64s} {s / 1e3:8.2f} {e / 1e3:8.2f} {(e - s) / 1e3:7.2f}")
tot = int(rows[i1 - 1]["End_Timestamp"]) - t0
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[i0:i1])
print(f"layer span {tot / 1e3:.2f} us, kernels {busy / 1e3:.2f} us")
