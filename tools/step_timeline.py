"""Print one timed outer iteration from a rocprofv3 kernel trace (the
(K-8)-th chained pass B to the next one) and the per-kernel stats.
  python tools/step_timeline.py gpurun_out/<tag>/prof/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_rowapply<17, 8, false" in r["Kernel_Name"]]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 8
i0, i1 = idx[-back], idx[-back + 1]
prev = int(rows[i0]["End_Timestamp"])
for r in rows[i0 + 1:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-62s dur %7.1f gap %6.1f" % (r["Kernel_Name"][:62], (e - s) / 1e3, (s - prev) / 1e3))
    prev = e
print("step %.1f us" % ((int(rows[i1]["End_Timestamp"]) - int(rows[i0]["End_Timestamp"])) / 1e3))
