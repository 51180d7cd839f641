#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per dispatch.

Conventions (/opt/skills/guides/MI355X_MICROARCH.md, "HBM" section):
  * rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch;
  * on gfx950 FETCH_SIZE counts exactly half of the bytes of a wide (16 B/lane) coalesced
    streaming read, so read bytes = 2 x FETCH_SIZE x 1024;
  * WRITE_SIZE is exact for 16 B/lane streaming stores: write bytes = WRITE_SIZE x 1024.
Every kernel of this library streams with 16 B/lane loads and stores (double2), so both
corrections apply.  The JSON written here is what bench.py reports as roofline.traffic.

usage: tools/pmc_summary.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <out.json> [label] [n_global,m,k,gpus]
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            acc[name].append(float(row["Counter_Value"]))
    return acc


def short(name):
    s = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return s.split("(")[0]


def main():
    fdir, wdir, out = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    workload = None
    if len(sys.argv) > 5:
        n, m, k, g = (int(float(v)) for v in sys.argv[5].split(","))
        workload = {"n_global": n, "roots": m, "qspace": k, "n_gpus": g}
    fetch = per_kernel(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for name in sorted(set(fetch) | set(write)):
        fv, wv = fetch.get(name, []), write.get(name, [])
        rd = 2.0 * 1024.0 * (sum(fv) / len(fv)) if fv else None
        wr = 1024.0 * (sum(wv) / len(wv)) if wv else None
        res[short(name)] = {
            "dispatches": max(len(fv), len(wv)),
            "read_bytes_per_dispatch": rd,
            "write_bytes_per_dispatch": wr,
            "hbm_bytes_per_dispatch": (rd or 0.0) + (wr or 0.0),
            "raw_fetch_kib_avg": sum(fv) / len(fv) if fv else None,
            "raw_write_kib_avg": sum(wv) / len(wv) if wv else None,
        }
    json.dump({"label": label, "workload": workload, "corrections": "read = 2 x FETCH_SIZE KiB x 1024; write = WRITE_SIZE KiB x 1024",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:40s} n={v['dispatches']:4d} read={v['read_bytes_per_dispatch'] or 0:.4g} "
              f"write={v['write_bytes_per_dispatch'] or 0:.4g}")


if __name__ == "__main__":
    main()
