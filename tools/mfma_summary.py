#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc pass of the MFMA counters into per-kernel matrix-core figures.

Counters (one pass: 3 SQ + 1 GRBM, within the per-pass limits of MI355X_MICROARCH.md):
  MfmaUtil      derived: sum(SQ_VALU_MFMA_BUSY_CYCLES) / (max(GRBM_GUI_ACTIVE) x SIMD_NUM) x 100
  MfmaFlopsF64  derived: SQ_INSTS_VALU_MFMA_MOPS_F64 x 512
  SQ_INSTS_VALU_MFMA_F64  MFMA f64 instructions issued
MFMA f64 rate = MfmaFlopsF64 / kernel duration (the dispatch's own timestamps), against the dense
f64 matrix peak of 78.6 TFLOP/s (MI355X spec).

usage: tools/mfma_summary.py <pmc dir> <out.json> [label]
"""
import csv
import json
import sys
from collections import defaultdict

PEAK_F64_TFLOPS = 78.6


def short(name):
    s = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return s.split("(")[0]


def main():
    pdir, out = sys.argv[1:3]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    vals = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    dur = defaultdict(dict)
    with open(f"{pdir}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            k, d = short(row["Kernel_Name"]), int(row["Dispatch_Id"])
            vals[k][d][row["Counter_Name"]] = float(row["Counter_Value"])
            dur[k][d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    res = {}
    for k, ds in vals.items():
        n = len(ds)
        flops = sum(v.get("MfmaFlopsF64", 0.0) for v in ds.values()) / n
        util = sum(v.get("MfmaUtil", 0.0) for v in ds.values()) / n
        insts = sum(v.get("SQ_INSTS_VALU_MFMA_F64", 0.0) for v in ds.values()) / n
        t = sum(dur[k].values()) / n
        if flops == 0 and insts == 0:
            continue
        res[k] = {
            "dispatches": n,
            "mfma_util_pct": round(util, 3),
            "mfma_f64_insts_per_dispatch": insts,
            "mfma_f64_flops_per_dispatch": flops,
            "avg_duration_us": round(t * 1e6, 2),
            "mfma_f64_tflops": round(flops / t / 1e12, 3) if t > 0 else None,
            "frac_of_f64_mfma_peak": round(flops / t / 1e12 / PEAK_F64_TFLOPS, 4) if t > 0 else None,
        }
    json.dump({"label": label, "peak_f64_mfma_tflops": PEAK_F64_TFLOPS, "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:36s} n={v['dispatches']:4d} util={v['mfma_util_pct']:7.3f}% "
              f"{v['mfma_f64_tflops']} TF/s ({v['frac_of_f64_mfma_peak']} of peak) t={v['avg_duration_us']} us")


if __name__ == "__main__":
    main()
