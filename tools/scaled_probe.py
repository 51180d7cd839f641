#!/usr/bin/env python3
"""A/B of the deferred-scal kernel instances (include/subspace_hip.h *_scaled) against the unscaled
ones on the same vectors at N = 1e8: gemm_inner 8x48 and 8x8 (symmetric), gemm_outer 48->8 (read-
modify-write), gemm_outer_set 48->8, axpy, dot.  Scales of 1 + 2^-20 force the SC instances; the
bytes and the call structure are identical.  Times are the library's HIP-event ledger, alternating
unscaled / scaled reps so that placement and clocks affect both alike.

usage: python tools/scaled_probe.py [--n 1e8] [--reps 6] [--out gpurun_out/scaled_probe.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))

import subspace_hip as sh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "scaled_probe.json"))
    a = ap.parse_args()
    n = int(a.n)
    ctx = sh.Context(0)
    pool = [ctx.alloc(n) for _ in range(64)]
    for i, v in enumerate(pool):
        ctx.fill_random(v, 9, i)
    rng = np.random.default_rng(0)
    s = 1.0 + 2.0 ** -20
    ones = np.ones(64)
    sc = np.full(64, s)
    al = rng.uniform(-1e-3, 1e-3, (48, 8))
    X, Y, R, O = pool[8:56], pool[:8], pool[56:64], pool[56:64]
    cases = {
        "gemm_inner 8x48": (lambda f: ctx.gemm_inner_scaled(Y, f[:8], X, f[:48]), 8.0 * n * 56),
        "gemm_inner 8x8 sym": (lambda f: ctx.gemm_inner_scaled(Y, f[:8], Y, f[:8]), 8.0 * n * 8),
        "gemm_outer 48->8": (lambda f: ctx.gemm_outer_scaled(al, X, f[:48], Y, f[:8]), 8.0 * n * 64),
        "gemm_outer_set 48->8": (lambda f: ctx.gemm_outer_set_scaled(al, X, f[:48], O), 8.0 * n * 56),
        "axpy": (lambda f: ctx.axpy_scaled(1e-3, X[0], f[0], Y[0], f[1]), 24.0 * n),
        "dot": (lambda f: ctx.dot_scaled(X[0], f[0], X[1], f[1]), 16.0 * n),
    }
    res = {}
    for name, (fn, nbytes) in cases.items():
        t = {"unscaled": [], "scaled": []}
        for r in range(a.reps + 1):
            for label, f in (("unscaled", ones), ("scaled", sc)):
                ctx.synchronize()
                ctx.ledger_reset()
                ctx.ledger_enable(True)
                fn(f)
                ctx.synchronize()
                led = ctx.ledger()
                ctx.ledger_enable(False)
                if r:
                    t[label].append(sum(v["ms"] for v in led.values()))
        row = {k: {"ms_median": float(np.median(v)), "GBs": nbytes / 1e6 / float(np.median(v))} for k, v in t.items()}
        row["scaled_over_unscaled"] = row["scaled"]["ms_median"] / row["unscaled"]["ms_median"]
        res[name] = row
        print(f"{name:22s} unscaled {row['unscaled']['GBs']:7.1f} GB/s  scaled {row['scaled']['GBs']:7.1f} GB/s  "
              f"ratio {row['scaled_over_unscaled']:.3f}", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"n": n, "reps": a.reps, "cases": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
