"""summary of one tools/gpu_iter.sh run: bench line + top kernels"""
import csv
import json
import sys

tag = sys.argv[1]
for ln in open(f"gpurun_out/b_{tag}.log"):
    if ln.startswith('{"metric"'):
        d = json.loads(ln)
        print(d["value"], d["stage_ms_per_step_rank0"], d.get("roofline", {}).get("avg_launch_us"))
rows = list(csv.DictReader(open(f"gpurun_out/px_{tag}/run_kernel_stats.csv")))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:80]}")
