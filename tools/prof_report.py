"""Summarise the rocprofv3 passes of tools/profile_round.sh into one JSON.

Per kernel: calls, average duration (kernel-trace stats), HBM bytes per
launch from the PMC passes, corrected as MI355X_MICROARCH.md prescribes for
gfx950: FETCH_SIZE (KB) counts half the bytes of a wide coalesced streaming
read -> x2; WRITE_SIZE (KB) is exact for 16 B/lane stores; and for the MFMA
kernels (mfma/ pass): MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (rocprofv3's MfmaUtil expression;
GRBM_GUI_ACTIVE is summed over the 8 XCDs), MFMA FLOPs = 512 x
SQ_INSTS_VALU_MFMA_MOPS_{F16,F32,I8} (the counters count ops / 512), and
TFLOP/s = those FLOPs / the kernel's average duration from the stats pass.
usage: python tools/prof_report.py <dir with stats/ fetch/ write/ mfma/>
"""
import collections
import csv
import glob
import json
import sys


def _csv(d, pat):
    f = glob.glob(f"{d}/**/{pat}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def pmc(d, sub, counter, scale=1024.0):
    acc = collections.defaultdict(list)
    for r in _csv(f"{d}/{sub}", "*counter_collection.csv"):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * scale)
    return {k: sum(v) / len(v) for k, v in acc.items()}


SIMDS, XCDS = 1024, 8   # MI355X: 256 CUs x 4 SIMDs, 8 XCDs


def main(d):
    stats = _csv(f"{d}/stats", "*kernel_stats.csv")
    fetch = pmc(d, "fetch", "FETCH_SIZE")
    write = pmc(d, "write", "WRITE_SIZE")
    busy = pmc(d, "mfma", "SQ_VALU_MFMA_BUSY_CYCLES", 1.0)
    gui = pmc(d, "mfma", "GRBM_GUI_ACTIVE", 1.0)
    mops = [pmc(d, "mfma", f"SQ_INSTS_VALU_MFMA_MOPS_{t}", 512.0) for t in ("F16", "F32", "I8")]
    tot = sum(float(r["TotalDurationNs"]) for r in stats) or 1.0
    out = {"kernels": [], "total_kernel_ms": round(tot / 1e6, 3),
           "notes": "avg_us from --kernel-trace --stats; hbm_read_bytes = 2 x FETCH_SIZE (gfx950 half-count "
                    "correction), hbm_write_bytes = WRITE_SIZE, per launch; mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / "
                    "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); mfma_flops = 512 x SQ_INSTS_VALU_MFMA_MOPS_{F16,F32,I8} "
                    "per launch; mfma_tflops = mfma_flops / avg_us"}
    for r in stats:
        name = r["Name"]
        k = {"name": name, "calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 3),
             "total_ms": round(float(r["TotalDurationNs"]) / 1e6, 3), "pct": round(float(r["Percentage"]), 2)}
        if name in fetch:
            k["hbm_read_bytes"] = round(2.0 * fetch[name])
        if name in write:
            k["hbm_write_bytes"] = round(write[name])
        if name in busy and gui.get(name):
            k["mfma_util"] = round(busy[name] / (gui[name] / XCDS * SIMDS), 4)
            fl = sum(m.get(name, 0.0) for m in mops)
            k["mfma_flops"] = fl
            k["mfma_tflops"] = round(fl / (float(r["AverageNs"]) * 1e-9) / 1e12, 1) if float(r["AverageNs"]) > 0 else None
        out["kernels"].append(k)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
