"""GPU idle gaps in a rocprofv3 kernel trace (run_kernel_trace.csv): span,
busy time, and the gaps above a threshold aggregated by the kernel that
follows them.  usage: trace_gaps.py TRACE.csv [threshold_us] [t_from_ms]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 5e3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
if len(sys.argv) > 3:
    rows = [r for r in rows if int(r["Start_Timestamp"]) - t0 >= float(sys.argv[3]) * 1e6]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
span = max(int(r["End_Timestamp"]) for r in rows) - int(rows[0]["Start_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
prev = int(rows[0]["End_Timestamp"])
for r in rows[1:]:
    st = int(r["Start_Timestamp"])
    g = st - prev
    if g > thr:
        a = agg[r["Kernel_Name"][:70]]
        a[0] += 1
        a[1] += g / 1e3
    prev = max(prev, int(r["End_Timestamp"]))
print("span %.2f ms busy %.2f ms (%.1f%%), %d kernels" % (span / 1e6, busy / 1e6, 100.0 * busy / span, len(rows)))
for k, (c, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:15]:
    print("  %6.1f us in %4d gaps before %s" % (us, c, k))
