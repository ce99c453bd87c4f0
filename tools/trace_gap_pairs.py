"""GPU idle gaps of a rocprofv3 kernel trace aggregated by (kernel before, kernel
after), over the part of the trace after t_from (fraction of the span).
usage: trace_gap_pairs.py TRACE.csv [min_us] [max_us] [t_from_frac]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
frac = float(sys.argv[4]) if len(sys.argv) > 4 else 0.3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in rows)
rows = [r for r in rows if int(r["Start_Timestamp"]) - t0 >= frac * (t1 - t0)]
agg = collections.defaultdict(lambda: [0, 0.0])
prev_end = int(rows[0]["End_Timestamp"])
prev_name = rows[0]["Kernel_Name"]
short = lambda s: s.replace("void cal::", "").replace("cal::", "").split("(")[0][:40]
for r in rows[1:]:
    g = (int(r["Start_Timestamp"]) - prev_end) / 1e3
    if lo < g <= hi:
        a = agg[(short(prev_name), short(r["Kernel_Name"]))]
        a[0] += 1
        a[1] += g
    if int(r["End_Timestamp"]) > prev_end:
        prev_end = int(r["End_Timestamp"])
        prev_name = r["Kernel_Name"]
tot = sum(v[1] for v in agg.values())
print("gaps in (%g, %g] us: %.2f ms" % (lo, hi, tot / 1e3))
for (a, b), (c, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print("  %7.1f us %4d x  %-40s -> %s" % (us, c, a, b))
