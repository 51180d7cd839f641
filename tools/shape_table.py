#!/usr/bin/env python3
"""One-page per-shape table of the C4-shard solve from ONE process: the solver ledger with
SSP_LEDGER_DETAIL=1 (one row per op and panel shape) and SSP_LEDGER_TIMING=dispatch (each op timed
from its first kernel's start to its last kernel's end, hipExtLaunchKernel events), run under
`rocprofv3 --kernel-trace`; the trace's last solve, summed per kernel instance, checks the ledger's
times (each ledger group against the kernel instances it launches).

usage: python tools/shape_table.py LEDGER.json RUN_kernel_trace.csv [--config C4-shard] > table.md
"""
import argparse
import collections
import csv
import json
import re

import numpy as np

# ledger row (regex on "op [tag]") -> kernel instances it launches (regex on the trace's names);
# the fold passes (k_reduce_publish / k_reduce_partials) of gemm_inner and transform_gram are counted
# with their op in the ledger and listed on their own in the trace.
GROUPS = [
    (r"^gemm_inner \[mfma-pre<2,(\d+)> .* sc\]", lambda m: rf"^k_gemm_inner<2, {m.group(1)}, false, true, \w+, true>"),
    (r"^gemm_inner \[sym<2,2> 8x8\]", lambda m: r"^k_gemm_inner<2, 2, true, false"),
    (r"^gemm_inner \[sym<2,2> 8x8 sc\]", lambda m: r"^k_gemm_inner<2, 2, true, true"),
    (r"^gemm_outer_set \[arg<8,1> \d+x8 sc\]", lambda m: r"^k_gemm_outer<8, false, true, true>"),
    (r"^gemm_outer_set \[arg<8,1> \d+x8\]", lambda m: r"^k_gemm_outer<8, false, true, false>"),
    (r"^gemm_outer \[arg<8,0> \d+x8 sc\]", lambda m: r"^k_gemm_outer<8, false, false, true>"),
    (r"^transform_gram \[transform<8,2> 8x8 sc\]", lambda m: r"^k_transform<8, 2, true>"),
    (r"^transform_gram \[transform<8,1> 8x8\]", lambda m: r"^k_transform<8, 1, true>"),
    (r"^axpy_pairs_norm$", lambda m: r"^k_axpy_pairs_norm"),
    (r"^precondition$", lambda m: r"^k_precondition"),
    (r"^p?_?action\(synthetic\)$", lambda m: r"^k_synth_(apply|coeff)"),
    (r"^fill$", lambda m: r"^k_fill"),
    (r"^scal$", lambda m: r"^k_scal\b"),
    (r"^select$", lambda m: r"^k_select_local"),
]


def short(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([\w:]+(<[^()]*>)?)", k)
    return m.group(1) if m else k


def last_solve(rows, first):
    """The kernels from the last launch of `first` (the solve's first kernel: the synthetic problem
    builds its diagonal once per solve) to the end of the trace."""
    ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    starts = [i for i, t in enumerate(ts) if t[2].startswith(first)]
    return ts[starts[-1]:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ledger")
    ap.add_argument("trace")
    ap.add_argument("--config", default="C4-shard")
    ap.add_argument("--first", default="k_synth_diag", help="the kernel each solve starts with")
    a = ap.parse_args()
    led = next(c for c in json.load(open(a.ledger)) if c["config"] == a.config)
    ops = {k: v for k, v in led["ops"].items() if v["calls"]}
    solve = last_solve(list(csv.DictReader(open(a.trace))), a.first)
    per_kernel = collections.defaultdict(lambda: [0, 0.0])
    for b, e, nm in solve:
        per_kernel[nm][0] += 1
        per_kernel[nm][1] += (e - b) / 1e3
    kern_total = sum(v[1] for v in per_kernel.values())
    wall = (solve[-1][1] - solve[0][0]) / 1e3
    led_total = sum(v["ms"] for v in ops.values()) * 1e3
    gb_total = sum(v["GB"] for v in ops.values())

    print(f"# {a.config}: per-shape table (N = {led['n']:,}, {led['iterations']} iterations)\n")
    print(f"One process: `tools/solver_ledger.py --configs {a.config}` with `SSP_LEDGER_DETAIL=1 "
          f"SSP_LEDGER_TIMING=dispatch` under `rocprofv3 --kernel-trace`; the ledger's second (warm) solve and "
          f"the trace's last solve are the same solve.\n")
    print(f"Ledger: {gb_total:.1f} GB algorithmic in {led_total / 1e3:.3f} ms of op time = "
          f"{gb_total / (led_total / 1e6) / 1e3:.2f} TB/s.  Trace: {len(solve)} kernels, {kern_total / 1e3:.3f} ms "
          f"of kernel time in a {wall / 1e3:.3f} ms window.\n")
    print("| op [instance, m×k, scaled] | calls | GB / call | µs / call | TB/s | share of op time |")
    print("|---|---:|---:|---:|---:|---:|")
    for k, v in sorted(ops.items(), key=lambda kv: -kv[1]["ms"]):
        us = 1e3 * v["ms"] / v["calls"]
        tbs = v["GB"] / (v["ms"] / 1e3) / 1e3 if v["ms"] and v["GB"] >= 0.05 else float("nan")
        print(f"| {k} | {v['calls']} | {v['GB'] / v['calls']:.3f} | {us:.1f} | "
              f"{'' if np.isnan(tbs) else f'{tbs:.2f}'} | {1e3 * v['ms'] / led_total:.3f} |")
    print("\n## Check against the trace (same solve)\n")
    print("| ledger rows | ms (ledger) | kernel instances | calls | ms (trace) | trace / ledger |")
    print("|---|---:|---|---:|---:|---:|")
    used = set()
    for lrx, krx_of in GROUPS:
        rows = {}
        for k, v in ops.items():
            m = re.match(lrx, k)
            if m:
                rows.setdefault(krx_of(m), []).append((k, v))
        for krx, lst in rows.items():
            lms = sum(v["ms"] for _, v in lst)
            kn = [nm for nm in per_kernel if re.match(krx, nm.replace("(anonymous namespace)::", ""))]
            used.update(kn)
            kms = sum(per_kernel[nm][1] for nm in kn) / 1e3
            kc = sum(per_kernel[nm][0] for nm in kn)
            label = lst[0][0] if len(lst) == 1 else f"{len(lst)} rows like {lst[0][0]}"
            print(f"| {label} | {lms:.3f} | {', '.join(sorted(kn)) or '-'} | {kc} | {kms:.3f} | "
                  f"{kms / lms if lms else float('nan'):.3f} |")
    rest = sorted(((nm, c) for nm, c in per_kernel.items() if nm not in used), key=lambda kv: -kv[1][1])
    print("\nOther kernels of the solve (fold passes, uploads, sparse terms): " +
          "; ".join(f"{nm} {c[0]}× {c[1] / 1e3:.3f} ms" for nm, c in rest))


if __name__ == "__main__":
    main()
