#!/usr/bin/env python3
"""Where the device's idle time goes in a solve (development tool): from a rocprofv3 --hip-trace
--kernel-trace pair, for every gap between consecutive kernels of the last solve, the host's part
(from the end of the previous kernel to the API call that launched the next one) and the launch part
(from that call to the kernel's start).  Usage: python tools/host_gap_analysis.py DIR [--split-gap-ms 5]
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--split-gap-ms", type=float, default=5.0)
    ap.add_argument("--min-gap-us", type=float, default=5.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    api = {}
    with open(os.path.join(a.dir, "run_hip_api_trace.csv")) as f:
        for r in csv.DictReader(f):
            api[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
    ks = []
    with open(os.path.join(a.dir, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Correlation_Id"])))
    ks.sort()
    start = 0
    for i in range(1, len(ks)):
        if ks[i][0] - ks[i - 1][1] > a.split_gap_ms * 1e6:
            start = i
    ks = ks[start:]
    host = launch = other = 0.0
    by_prev = defaultdict(lambda: [0, 0.0, 0.0])
    ngaps = 0
    for (s0, e0, n0, c0), (s1, e1, n1, c1) in zip(ks, ks[1:]):
        gap = (s1 - e0) / 1e3
        if gap < a.min_gap_us:
            other += max(0.0, gap)
            continue
        ngaps += 1
        t_api = api.get(c1, (s1, s1, "?"))[0]
        h = max(0.0, (t_api - e0) / 1e3)
        h = min(h, gap)
        l = gap - h
        host += h
        launch += l
        k = re.sub(r"\(.*", "", re.sub(r"^void ", "", n0).replace("(anonymous namespace)::", ""))[:50]
        by_prev[k][0] += 1
        by_prev[k][1] += h
        by_prev[k][2] += l
    busy = sum((e - s) for s, e, _, _ in ks) / 1e3
    wall = (ks[-1][1] - ks[0][0]) / 1e3
    out = {"dispatches": len(ks), "wall_us": round(wall, 1), "busy_us": round(busy, 1),
           "idle_us": round(wall - busy, 1), "gaps_over_min": ngaps,
           "host_part_us": round(host, 1), "launch_part_us": round(launch, 1), "short_gaps_us": round(other, 1),
           "after": {k: {"gaps": v[0], "host_us": round(v[1], 1), "launch_us": round(v[2], 1)}
                     for k, v in sorted(by_prev.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:15]}}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
