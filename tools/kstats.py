"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in rows[:top]:
    print("%-64s %6s %9.2f ms %9.1f us" % (r["Name"][:64], r["Calls"], int(r["TotalDurationNs"]) / 1e6,
                                           float(r["AverageNs"]) / 1e3))
