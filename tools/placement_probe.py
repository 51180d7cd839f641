#!/usr/bin/env python3
"""Why do the same panel shapes stream slower inside the C4-shard solve than in the per-shape bench?
(development probe).  One process, one context: the C4 shapes on a fresh vector pool, then two
C4-shard solves (the arena churns: the Q space prepends and drops vectors), then the same shapes on
a pool allocated from the arena's cached blocks afterwards -- and again after freeing that pool in a
shuffled order.  Times are the library's HIP-event ledger.

usage: python tools/placement_probe.py --out gpurun_out/placement.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402
from solver_ledger import CONFIGS  # noqa: E402

N = 12_500_000


def shapes(ctx, pool, reps, tag):
    s = 1.0 + 2.0 ** -20
    sc = np.full(80, s)
    al = np.random.default_rng(0).uniform(-1e-3, 1e-3, (48, 8))
    cases = [
        ("gemm_inner 8x16 sc", "gemm_inner", lambda: ctx.gemm_inner_scaled(pool[:8], sc[:8], pool[8:24], sc[:16]), 24),
        ("gemm_inner 8x40 sc", "gemm_inner", lambda: ctx.gemm_inner_scaled(pool[:8], sc[:8], pool[8:48], sc[:40]), 48),
        ("gemm_inner 8x56 sc", "gemm_inner", lambda: ctx.gemm_inner_scaled(pool[:8], sc[:8], pool[8:64], sc[:56]), 64),
        ("gemm_outer_set 48->8", "gemm_outer_set", lambda: ctx.gemm_outer_set_scaled(al, pool[8:56], sc[:48], pool[64:72]), 56),
    ]
    out = {}
    for name, op, fn, nvec in cases:
        fn()
        ctx.synchronize()
        ctx.ledger_reset()
        ctx.ledger_enable(True)
        for _ in range(reps):
            fn()
        ctx.synchronize()
        e = ctx.ledger()[op]
        ctx.ledger_enable(False)
        us = 1e3 * e["ms"] / e["calls"]
        out[name] = round(8.0 * N * nvec / (us * 1e-6) / 1e9, 1)
        print(f"{tag:10s} {name:22s} {us:9.1f} us {out[name]:8.1f} GB/s", flush=True)
    return out


def solve(ctx, tag):
    solver, n, kw = CONFIGS["C4-shard"]
    kw = dict(kw)
    rho, rank, seed = kw.pop("rho"), kw.pop("rank"), kw.pop("seed")
    ctx.ledger_reset()
    ctx.ledger_enable(True)
    ih.davidson_synthetic(ctx, n, rho, rank, seed, n_local=0, **kw)
    ctx.ledger_enable(False)
    led = ctx.ledger()
    ms = sum(v["ms"] for v in led.values())
    nb = sum(v["bytes"] for v in led.values())
    res = {"kernel_ms": round(ms, 3), "kernel_GBs": round(nb / ms / 1e6, 1),
           "ops": {op: round(v["bytes"] / v["ms"] / 1e6, 1) for op, v in led.items() if v["ms"] > 0.5}}
    print(f"{tag:10s} solve kernel {ms:.3f} ms {res['kernel_GBs']} GB/s {res['ops']}", flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ctx = sh.Context(0)
    res = {}
    pool = [ctx.alloc(N) for _ in range(72)]
    for i, v in enumerate(pool):
        ctx.fill_random(v, 5, i)
    res["fresh"] = shapes(ctx, pool, a.reps, "fresh")
    for v in pool:
        v.free()
    res["solve1"] = solve(ctx, "solve1")
    res["solve2"] = solve(ctx, "solve2")
    pool = [ctx.alloc(N) for _ in range(72)]
    for i, v in enumerate(pool):
        ctx.fill_random(v, 5, i)
    res["after_solve"] = shapes(ctx, pool, a.reps, "after")
    order = np.random.default_rng(1).permutation(len(pool))
    for i in order:
        pool[i].free()
    pool = [ctx.alloc(N) for _ in range(72)]
    for i, v in enumerate(pool):
        ctx.fill_random(v, 5, i)
    res["shuffled"] = shapes(ctx, pool, a.reps, "shuffled")
    res["solve3"] = solve(ctx, "solve3")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
