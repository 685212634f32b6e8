"""Sum rocprofv3 counter_collection.csv files per dispatch (kernel name + counters)."""
import collections
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("__amd"):
            continue
        k = r["Kernel_Name"][:50] + " #" + r["Dispatch_Id"]
        agg.setdefault(k, collections.OrderedDict())
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, v in agg.items():
        print(k, " ".join(f"{a}={b:.4g}" for a, b in v.items()))
