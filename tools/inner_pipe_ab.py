#!/usr/bin/env python3
"""gemm_inner per-shape rates at the C4 shard's length (12.5e6 elements), scaled and unscaled, for
the A/B of the two-stage load loop (k_gemm_inner PIPE, SSP_INNER_PIPE=0/1/2 -- set by the caller,
read once per process).  Times are the library's HIP-event ledger; bytes the algorithmic bytes (every
distinct vector of the panel read once).

usage: SSP_INNER_PIPE=1 python tools/inner_pipe_ab.py [--n 12.5e6] [--reps 8] --out gpurun_out/x.json
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
    ap.add_argument("--n", type=float, default=12.5e6)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    n = int(a.n)
    ctx = sh.Context(0)
    pool = [ctx.alloc(n) for _ in range(72)]
    for i, v in enumerate(pool):
        ctx.fill_random(v, 11, i)
    s = 1.0 + 2.0 ** -20
    sc = np.full(72, s)
    cases = []
    for k in (4, 8, 11, 12, 16, 20, 24, 32, 40, 48, 64):
        cases.append((f"8x{k} scaled", lambda k=k: ctx.gemm_inner_scaled(pool[:8], sc[:8], pool[8:8 + k], sc[:k]),
                      8.0 * n * (8 + k)))
    for k in (16, 40, 48):
        cases.append((f"8x{k}", lambda k=k: ctx.gemm_inner(pool[:8], pool[8:8 + k]), 8.0 * n * (8 + k)))
    # as in the solver: the rows were just rewritten (precondition / orthonormalisation, 8 vectors
    # read-modify-write) before the overlap reads them; only the gemm_inner is timed
    for k in (8, 16, 32, 48):
        def pre(k=k):
            for v in pool[:8]:
                ctx.scal(0.9999999, v)
            return ctx.gemm_inner_scaled(pool[:8], sc[:8], pool[8:8 + k], sc[:k])
        cases.append((f"8x{k} sc after rmw", pre, 8.0 * n * (8 + k)))
    cases.append(("8x8 sym", lambda: ctx.gemm_inner(pool[:8], pool[:8]), 8.0 * n * 8))
    cases.append(("8x8 sym scaled", lambda: ctx.gemm_inner_scaled(pool[:8], sc[:8], pool[:8], sc[:8]), 8.0 * n * 8))
    res = {}
    for name, fn, nbytes in cases:
        fn()
        ctx.synchronize()
        ctx.ledger_reset()
        ctx.ledger_enable(True)
        for _ in range(a.reps):
            fn()
        ctx.synchronize()
        led = ctx.ledger()
        ctx.ledger_enable(False)
        e = led["gemm_inner"]
        us = 1e3 * e["ms"] / e["calls"]
        res[name] = {"avg_us": round(us, 2), "GBs": round(nbytes / (us * 1e-6) / 1e9, 1), "bytes": nbytes}
        print(f"pipe={os.environ.get('SSP_INNER_PIPE', '1')} {name:18s} {us:9.1f} us {res[name]['GBs']:8.1f} GB/s",
              flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump({"n": n, "reps": a.reps, "pipe": os.environ.get("SSP_INNER_PIPE", "1"), "cases": res},
              open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
