#!/usr/bin/env python3
"""Does an idle gap before a launch slow the launch down?  Times (HIP-event ledger) gemm_inner 8 x 72
and gemm_outer_set 48 -> 8 at the C4 shard length (1.25e7) and at N = 1e8 when they follow each other
at once, and after the host has left the GPU idle for 0.02 / 0.2 / 2 ms (the solve's round trips and
host algebra leave gaps of that size).  Development probe; prints one JSON line per case.

usage: python tools/gap_probe.py [--out gpurun_out/gap_probe.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402


def spin(seconds):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        pass


def run(ctx, n, m, k, reps, gap_s):
    xs = [ctx.alloc(n) for _ in range(m)]
    ys = [ctx.alloc(n) for _ in range(k)]
    for i, v in enumerate(xs + ys):
        ctx.fill(1.0 / (i + 1), v)
    alphas = np.random.default_rng(1).uniform(-1, 1, (k, m))
    out = {}
    for op in ("gemm_inner", "gemm_outer_set"):
        ctx.synchronize()
        ctx.ledger_reset()
        ctx.ledger_enable(True)
        for _ in range(reps):
            if gap_s is not None:
                ctx.synchronize()
                spin(gap_s)
            if op == "gemm_inner":
                ctx.gemm_inner(xs, ys)
            else:
                ctx.gemm_outer_set(alphas, ys, xs)
        ctx.synchronize()
        ctx.ledger_enable(False)
        led = ctx.ledger()
        e = led[op]
        out[op] = {"us_per_call": round(1e3 * e["ms"] / e["calls"], 1),
                   "GBs": round(e["bytes"] / (e["ms"] / 1e3) / 1e9, 1), "calls": e["calls"]}
    for v in xs + ys:
        v.free()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "gap_probe.json"))
    a = ap.parse_args()
    ctx = sh.Context(0)
    res = []
    for n, reps in ((12_500_000, 20), (100_000_000, 5)):
        for gap in (None, 2e-5, 2e-4, 2e-3):
            r = {"n": n, "m": 8, "k": 72 if n < 50_000_000 else 48, "gap_ms": None if gap is None else 1e3 * gap}
            r.update(run(ctx, n, 8, r["k"], reps, gap))
            print(json.dumps(r), flush=True)
            res.append(r)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
