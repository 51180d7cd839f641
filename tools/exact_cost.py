#!/usr/bin/env python3
"""Cost of the reference-arithmetic path on short vectors (development tool): per-call wall time of
dot, gemm_inner 8x48, gemm_outer 48->8 and axpy with ssp_ctx_set_exact_max on (sequential sums,
kernels_exact.hip) and off (the bandwidth kernels), and whole C1-sized solves either way.

usage: python tools/exact_cost.py [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))

import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402


def per_call(ctx, fn, reps):
    fn()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ctx = sh.Context(0)
    r = np.random.default_rng(1)
    out = {"unit": "us per call (host wall, synchronised)", "ops": {}, "solves": {}}
    for n in (1000, 2048, 4096, 16384):
        xs = [ctx.upload(r.uniform(-1, 1, n)) for _ in range(48)]
        ys = [ctx.upload(r.uniform(-1, 1, n)) for _ in range(8)]
        al = r.uniform(-1, 1, (48, 8))
        row = {}
        for mode, lim in (("exact", 16384), ("bandwidth", 0)):
            ctx.set_exact_max(lim)
            row[mode] = {
                "dot": per_call(ctx, lambda: ctx.dot(xs[0], xs[1]), 200),
                "gemm_inner_8x48": per_call(ctx, lambda: ctx.gemm_inner(ys, xs), 50),
                "gemm_outer_48to8": per_call(ctx, lambda: ctx.gemm_outer(al, xs, ys), 50),
                "axpy": per_call(ctx, lambda: ctx.axpy(0.5, xs[0], ys[0]), 200),
            }
        out["ops"][str(n)] = row
        print(n, json.dumps(row), flush=True)
        for v in xs + ys:
            v.free()
    for name, n, rank in (("C1_rank1", 10_000, 1), ("C1_rank8", 10_000, 8)):
        row = {}
        for mode, lim in (("exact", 16384), ("bandwidth", 0)):
            ctx.set_exact_max(lim)
            kw = dict(nroots=1, max_p=0, convergence_threshold=1e-8, max_size_qspace=6, reset_D=8)
            ih.davidson_synthetic(ctx, n, 0.1, rank, 1, solutions=False, **kw)
            t0 = time.perf_counter()
            g = ih.davidson_synthetic(ctx, n, 0.1, rank, 1, solutions=False, **kw)
            row[mode] = {"wall_ms": 1e3 * (time.perf_counter() - t0), "iterations": g["iterations"]}
        out["solves"][name] = row
        print(name, json.dumps(row), flush=True)
    ctx.set_exact_max(2048)
    ctx.close()
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
