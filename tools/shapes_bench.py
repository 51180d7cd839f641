#!/usr/bin/env python3
"""Per-shape microbenchmark of the handler ops at fixed N (SURVEY.md §8d "Concrete synthetic
inputs", shapes: gemm_inner 8x48, 8x1, 1x6; gemm_outer 48->8, 1->8, 6->1; axpy; dot ...).
Times come from the library's HIP-event ledger (events on the context stream around each op), one
ledger window per call: two warm-up calls, then the median (and mean) over --reps calls, as §8d
prescribes (median of 10 after 2 warm-ups); bytes are the algorithmic bytes of DESIGN.md §4.

usage: python tools/shapes_bench.py [--n 1e8] [--reps 10] [--out gpurun_out/shapes.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))

import subspace_hip as sh  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "shapes.json"))
    a = ap.parse_args()
    n = int(a.n)
    ctx = sh.Context(0)
    pool = [ctx.alloc(n) for _ in range(80)]
    for i, v in enumerate(pool):
        ctx.fill_random(v, 7, i)
    d = ctx.alloc(n)
    ctx.synthetic_diagonal(d, 0.1, 1)
    rng = np.random.default_rng(0)
    cases = []
    for m, k in ((8, 48), (8, 1), (1, 6), (1, 48), (4, 24), (16, 64), (48, 8), (1, 1), (1, 2), (2, 2), (1, 3)):
        cases.append((f"gemm_inner {m}x{k}", "gemm_inner",
                      lambda m=m, k=k: ctx.gemm_inner(pool[:m], pool[m:m + k])))
    # the same 8 x 48 panel on other vector sets: rows from the last-allocated vectors, and rows and
    # columns exchanged (role against placement)
    cases.append(("gemm_inner 8x48 rows=pool[48:56]", "gemm_inner", lambda: ctx.gemm_inner(pool[48:56], pool[0:48])))
    cases.append(("gemm_inner 8x48 rows=pool[8:16]", "gemm_inner", lambda: ctx.gemm_inner(pool[8:16], pool[16:64])))
    cases.append(("gemm_inner 8x48 rows=pool[0:8] again", "gemm_inner", lambda: ctx.gemm_inner(pool[:8], pool[8:56])))
    for k, m in ((48, 8), (1, 8), (6, 1), (8, 8), (24, 4), (64, 16)):
        al = rng.uniform(-0.1, 0.1, (k, m))
        cases.append((f"gemm_outer {k}->{m}", "gemm_outer",
                      lambda al=al, k=k, m=m: ctx.gemm_outer(al, pool[16:16 + k], pool[:m])))
    cases += [
        ("dot x.y", "dot", lambda: ctx.dot(pool[0], pool[1])),
        ("dot x.x", "dot", lambda: ctx.dot(pool[0], pool[0])),
        ("axpy", "axpy", lambda: ctx.axpy(1e-3, pool[1], pool[2])),
        ("scal", "scal", lambda: ctx.scal(0.999, pool[3])),
        ("copy", "copy", lambda: ctx.copy(pool[4], pool[5])),
        ("fill", "fill", lambda: ctx.fill(0.0, pool[6])),
        ("precondition x8", "precondition", lambda: ctx.precondition(pool[:8], d, [0.5] * 8)),
        ("select 16 (min)", "select", lambda: ctx.select(d, 16)),
    ]
    res = []
    for name, op, fn in cases:
        for _ in range(2):
            fn()
        ctx.synchronize()
        per_call, nbytes = [], 0.0
        for _ in range(a.reps):
            ctx.ledger_reset()
            ctx.ledger_enable(True)
            fn()
            ctx.ledger_enable(False)
            e = ctx.ledger()[op]
            per_call.append(e["ms"] / e["calls"])
            nbytes = e["bytes"] / e["calls"]
        med = float(np.median(per_call))
        us, mean_us = 1e3 * med, 1e3 * float(np.mean(per_call))
        gbs = nbytes / (med / 1e3) / 1e9
        res.append({"case": name, "median_us": round(us, 2), "mean_us": round(mean_us, 2), "bytes_per_call": nbytes,
                    "GBs": round(gbs, 1), "frac_of_8TBs": round(gbs / PEAK, 4)})
        print(f"{name:22s} {us:10.1f} us {gbs:8.1f} GB/s", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"n": n, "reps": a.reps, "cases": res}, open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
