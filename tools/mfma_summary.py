"""Summarise a rocprofv3 --pmc pass of SQ_INSTS_VALU_MFMA_MOPS_F64 /
SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE per kernel (with the kernel-trace
durations of the same command): MFMA f64 flops per launch (MOPS x 512, the
convention pinned in round 1: 512 n per Gram sweep of n rows), TFLOP/s
against the f64 matrix peak, and the MFMA-busy share of the kernel's
cycles.  usage: mfma_summary.py COUNTERS.csv KERNEL_STATS.csv OUT.json"""
import collections
import csv
import json
import sys

PEAK = 78.6
rows = list(csv.DictReader(open(sys.argv[1])))
stats = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(sys.argv[2]))}
per = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, c in per.items():
    mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", [0])
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])
    grbm = c.get("GRBM_GUI_ACTIVE", [0])
    sqb = c.get("SQ_BUSY_CYCLES", [0])
    n = len(mops)
    flops = 512.0 * sum(mops) / n
    avg_ns = stats.get(k)
    d = {"launches": n, "mfma_f64_flops_per_launch": flops,
         "mfma_busy_cycles_per_launch": sum(busy) / n, "grbm_gui_active_per_launch": sum(grbm) / n,
         "sq_busy_cycles_per_launch": sum(sqb) / n, "avg_launch_us_trace": avg_ns / 1e3 if avg_ns else None}
    if avg_ns:
        d["tflops"] = flops / (avg_ns * 1e-9) / 1e12
        d["frac_of_f64_matrix_peak"] = d["tflops"] / PEAK
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md §DVFS);
    # MFMA busy cycles over the 1024 SIMDs
    if grbm and sum(grbm) > 0:
        d["mfma_busy_share"] = (sum(busy) / n / 1024.0) / (sum(grbm) / n / 8.0)
    out[k] = d
json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
for k, d in sorted(out.items(), key=lambda x: -x[1]["mfma_f64_flops_per_launch"])[:12]:
    print("%-70s n=%3d flops %.3e tf %s busy %s" % (k[:70], d["launches"], d["mfma_f64_flops_per_launch"],
                                                  round(d.get("tflops", 0), 1), round(d.get("mfma_busy_share", 0), 3)))
