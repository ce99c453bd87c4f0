"""Per-launch HBM traffic of the bench's kernels from rocprofv3 --pmc CSVs.

  python tools/traffic_json.py gpurun_out/pmc [--out profiles/spmv_traffic.json]

Reads <dir>/bench_fetch/run_counter_collection.csv (FETCH_SIZE) and
<dir>/bench_write/run_counter_collection.csv (WRITE_SIZE), both in KiB.
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports
half the bytes of a coalesced streaming read, so it is doubled.  Writes one
JSON object per kernel class plus the entry bench.py reads (kernel "spmv").
"""
import argparse
import collections
import csv
import json
import os

CLASSES = {  # kernel-name prefix -> kernel
    "void cal::k_spmv_pair<1": "spmv",
    "void cal::k_spmv_planes<1": "spmv",
    "void cal::k_spmv_pat_lds<1": "spmv",
    "void cal::k_spmv<1": "spmv_csr",
    "void cal::k_rowapply<17, 4, true, false": "gram_p1",
    "void cal::k_rowapply<17, 8, true, true, false": "gram_passA",
    "void cal::k_rowapply<17, 8, false, true, true, true": "apply_passB",
}
# bench.py kernel classes (kernel_ms_per_step keys): per-launch average over members
BENCH_CLASSES = {"spmv": ["spmv"], "gram": ["gram_p1", "gram_passA"], "apply": ["apply_passB"]}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for pre, cls in CLASSES.items():
            if r["Kernel_Name"].startswith(pre):
                acc[cls].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--out", default="profiles/spmv_traffic.json")
    p.add_argument("--workload", default="lap3d_215")
    a = p.parse_args()
    fetch = per_kernel(os.path.join(a.dir, "bench_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.dir, "bench_write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = 2.0 * fetch.get(k, 0.0)
        w = write.get(k, 0.0)
        kernels[k] = {"fetch_bytes_x2": f, "write_bytes": w, "hbm_bytes_per_launch": f + w}
    classes = {}
    for cls, members in BENCH_CLASSES.items():
        vals = [kernels[m]["hbm_bytes_per_launch"] for m in members if m in kernels]
        if vals:
            classes[cls] = sum(vals) / len(vals)
    out = {"workload": a.workload, "n_gpus": 1, "classes": classes,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py; "
                     "FETCH_SIZE x2 (gfx950 streaming-read correction), KiB x 1024",
           "kernels": kernels}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
