"""Idle gaps on the busiest queue of a rocprofv3 csv trace (kernels and
copies), over the last SPAN ms of the run: the gaps sorted by size with the
launch before and after each.  Not part of the library.
    python tools/trace_idle.py DIR/run [SPAN_MS]"""
import csv
import sys


def main():
    base = sys.argv[1]
    span = float(sys.argv[2]) if len(sys.argv) > 2 else 30.0
    ev = []
    for suffix, name_key in (("_kernel_trace.csv", "Kernel_Name"), ("_memory_copy_trace.csv", "Direction")):
        try:
            for r in csv.DictReader(open(base + suffix)):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(name_key, "?")[:60],
                           r.get("Queue_Id", r.get("Stream_Id", "?"))))
        except FileNotFoundError:
            pass
    ev.sort()
    t_end = max(e[1] for e in ev)
    ev = [e for e in ev if e[0] >= t_end - span * 1e6]
    gaps, cur, prev_name = [], ev[0][1], ev[0][2]
    t0 = ev[0][0]
    for a, b, name, q in ev[1:]:
        if a > cur:
            gaps.append((a - cur, (cur - t0) / 1e3, prev_name, name))
        cur = max(cur, b)
        prev_name = name
    tot = (cur - t0) / 1e6
    g = sum(x[0] for x in gaps) / 1e6
    print("window %.3f ms, idle %.3f ms (%.1f%%), %d gaps" % (tot, g, 100 * g / tot, len(gaps)))
    for d, at, before, after in sorted(gaps, reverse=True)[:40]:
        print("%8.1f us at %8.3f ms  %-60s -> %s" % (d / 1e3, at / 1e3, before, after))


if __name__ == "__main__":
    main()
