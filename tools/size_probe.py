#!/usr/bin/env python3
"""Per-launch time against vector length: gemm_inner 8 x 48, gemm_outer_set 48 -> 8 and gemm_outer 48 -> 8
(RMW), transform_gram 8 x 8 and axpy_pairs_norm 8, at N = 1.5625e6 .. 1e8 (HIP-event ledger, 10 calls
each after 2 untimed), and the least-squares fit t = t0 + bytes / R per op: t0 is what a launch costs
beyond streaming its bytes (ramp, tail, the reduction's fold), R the streaming rate.  Development
probe; prints one JSON line per op and length.

usage: python tools/size_probe.py [--out gpurun_out/size_probe.json] [--ops gemm_inner,gemm_outer_set]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402

NS = (1_562_500, 3_125_000, 6_250_000, 12_500_000, 25_000_000, 50_000_000, 100_000_000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "size_probe.json"))
    ap.add_argument("--ops", default="gemm_inner,gemm_outer_set,gemm_outer,transform_gram,axpy_pairs_norm")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--ns", default=",".join(str(n) for n in NS), help="comma-separated lengths")
    a = ap.parse_args()
    ops = a.ops.split(",")
    m, k = 8, 48
    ctx = sh.Context(0)
    rng = np.random.default_rng(1)
    alphas = rng.uniform(-1, 1, (k, m)) / k
    t8 = np.eye(m) + rng.uniform(-1e-3, 1e-3, (m, m))
    res = []
    for n in (int(float(v)) for v in a.ns.split(",")):
        xs = [ctx.alloc(n) for _ in range(m)]
        ys = [ctx.alloc(n) for _ in range(k)]
        for i, v in enumerate(xs + ys):
            ctx.fill(1.0 / (i + 1), v)
        calls = {
            "gemm_inner": lambda: ctx.gemm_inner(xs, ys),
            "gemm_outer_set": lambda: ctx.gemm_outer_set(alphas, ys, xs),
            "gemm_outer": lambda: ctx.gemm_outer(alphas, ys, xs),
            "transform_gram": lambda: ctx.transform_gram(t8, xs),
            "axpy_pairs_norm": lambda: ctx.axpy_pairs_norm([0.5] * m, ys[:m], xs),
        }
        for op in ops:
            for _ in range(2):
                calls[op]()
            ctx.synchronize()
            ctx.ledger_reset()
            ctx.ledger_enable(True)
            for _ in range(a.reps):
                calls[op]()
            ctx.synchronize()
            ctx.ledger_enable(False)
            led = ctx.ledger()
            e = led[op]
            r = {"op": op, "n": n, "us": round(1e3 * e["ms"] / e["calls"], 2), "bytes": e["bytes"] / e["calls"],
                 "GBs": round(e["bytes"] / (e["ms"] / 1e3) / 1e9, 1)}
            print(json.dumps(r), flush=True)
            res.append(r)
        for v in xs + ys:
            v.free()
    fits = {}
    for op in ops:
        pts = [(r["bytes"], r["us"]) for r in res if r["op"] == op]
        b = np.array([p[0] for p in pts])
        t = np.array([p[1] for p in pts])
        A = np.vstack([np.ones_like(b), b]).T
        (t0, inv), *_ = np.linalg.lstsq(A, t, rcond=None)
        fits[op] = {"t0_us": round(float(t0), 1), "R_GBs": round(float(1e-3 / inv), 1)}
    print(json.dumps({"fits": fits}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"points": res, "fits": fits}, open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
