"""Per-step kernel timeline from a rocprofv3 kernel trace (tools/gpu_trace.sh):
the kernels between two consecutive launches of the step's first SpMV, with
their durations and the idle gaps.  python tools/trace_step.py TRACE.csv [marker]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "k_spmv_pair<1"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
starts = [i for i, x in enumerate(k) if marker in x[2]]
# the step begins at the first of the 8 consecutive SpMVs
steps = [i for j, i in enumerate(starts) if j == 0 or starts[j - 1] != i - 1]
a, b = steps[-3], steps[-2]
t0 = k[a][0]
prev = t0
tot_busy = 0
for s, e, name in k[a:b]:
    gap = s - prev
    print("%8.1f  %7.1f us  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, name[:110]))
    prev = max(prev, e)
    tot_busy += e - s
print("step %.1f us, busy %.1f us" % ((k[b][0] - t0) / 1e3, tot_busy / 1e3))
