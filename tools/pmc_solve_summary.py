#!/usr/bin/env python3
"""HBM traffic of a whole solve from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over
tools/solver_ledger.py (one config, `repeat` solves per process), against the library ledger's
algorithmic bytes of the same solve.  Corrections as tools/pmc_summary.py (MI355X_MICROARCH.md:
read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB, for 16 B/lane streaming accesses -- every
large kernel of the library; the small reduction / fix-up kernels move a few KiB).

usage: tools/pmc_solve_summary.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <solver_ledger.json> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def totals(path, counter):
    acc, cnt = defaultdict(float), defaultdict(int)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            acc[name] += float(row["Counter_Value"])
            cnt[name] += 1
    return acc, cnt


def main():
    fdir, wdir, ledger, out = sys.argv[1:5]
    fetch, nf = totals(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE")
    write, _ = totals(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE")
    led = json.load(open(ledger))[0]
    solves = 2  # tools/solver_ledger.py run(repeat=2): a cold and a warm solve in the profiled process
    kernels = {}
    for name in set(fetch) | set(write):
        rd = 2048.0 * fetch.get(name, 0.0) / solves
        wr = 1024.0 * write.get(name, 0.0) / solves
        kernels[name] = {"dispatches_per_solve": nf.get(name, 0) / solves, "read_GB": rd / 1e9, "write_GB": wr / 1e9}
    tot = sum(v["read_GB"] + v["write_GB"] for v in kernels.values())
    res = {
        "config": led["config"], "iterations": led["iterations"],
        "hbm_GB_per_solve_pmc": round(tot, 2),
        "algorithmic_GB_per_solve_ledger": led["algorithmic_GB"],
        "pmc_over_algorithmic": round(tot / led["algorithmic_GB"], 4),
        # plain scal passes (k_scal / k_scal_win; not the fused k_scal_inner) and copies per solve
        "scal_kernels_dispatched": sum(v["dispatches_per_solve"] for k, v in kernels.items()
                                       if k in ("k_scal", "k_scal_win")),
        "copy_kernels_dispatched": sum(v["dispatches_per_solve"] for k, v in kernels.items() if k.startswith("k_copy")),
        "corrections": "read = 2 x FETCH_SIZE KiB x 1024; write = WRITE_SIZE KiB x 1024",
        "kernels": dict(sorted(kernels.items(), key=lambda kv: -(kv[1]["read_GB"] + kv[1]["write_GB"]))),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
