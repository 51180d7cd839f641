#!/usr/bin/env python3
"""Idle-GPU gaps of a solve from a rocprofv3 --kernel-trace CSV (development tool).

The device is idle between the end of one kernel and the start of the next on the context's
stream; in a solve those gaps are the host round trips (a reduction's result travels to the host,
the host decides, the next kernels are launched) and launch spacing.  Groups the gaps by the kernel
that precedes them, over the dispatches of the last `--window` seconds of the trace (the warm solve
of tools/solver_ledger.py), and prints / writes the totals.

usage: python tools/gap_analysis.py run_kernel_trace.csv [--last-solve-ms 80] [--out gaps.json]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:60] or "?"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--span-ms", type=float, default=None,
                    help="analyse the dispatches of the last span (default: the whole trace)")
    ap.add_argument("--split-gap-ms", type=float, default=5.0,
                    help="a gap longer than this separates solves; the last solve is analysed")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the last solve: the dispatches after the last gap longer than split-gap-ms
    start = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > a.split_gap_ms * 1e6:
            start = i
    rows = rows[start:]
    if a.span_ms:
        t_end = rows[-1][1]
        rows = [r for r in rows if r[0] >= t_end - a.span_ms * 1e6]
    busy = sum(e - s for s, e, _ in rows)
    wall = rows[-1][1] - rows[0][0]
    after = defaultdict(lambda: [0, 0.0])
    hist = defaultdict(int)
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = max(0, s1 - e0)
        k = short(n0)
        after[k][0] += 1
        after[k][1] += g / 1e3
        b = "<2us" if g < 2e3 else "2-5us" if g < 5e3 else "5-10us" if g < 1e4 else "10-20us" if g < 2e4 else \
            "20-50us" if g < 5e4 else "50-100us" if g < 1e5 else ">100us"
        hist[b] += 1
    top = sorted(after.items(), key=lambda kv: -kv[1][1])
    out = {"dispatches": len(rows), "wall_ms": round(wall / 1e6, 3), "busy_ms": round(busy / 1e6, 3),
           "idle_ms": round((wall - busy) / 1e6, 3), "gap_histogram": dict(hist),
           "idle_after": {k: {"gaps": v[0], "us": round(v[1], 1), "us_per_gap": round(v[1] / max(1, v[0]), 2)}
                          for k, v in top[:25]}}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
