#!/usr/bin/env python3
"""ssp_transform_gram (the block self-orthonormalisation's pass) against the streaming kernels beside it,
by the HIP-event ledger: 8 vectors in place at N = 1e8 and 1.25e7 (one C4 shard), plain and with the fused
Gram matrix, and the symmetric 8 x 8 gemm_inner.  Development tool.

usage: python tools/transform_probe.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
out = {}
with sh.Context(0) as ctx:
    for n in (100_000_000, 12_500_000):
        for m in (8, 4):
            xs = [ctx.alloc(n) for _ in range(m)]
            for v, x in enumerate(xs):
                ctx.lib.sspx_fill_random(ctx.handle, x.ptr, n, 0, 7, v)
            t = np.triu(np.full((m, m), 1e-3)) + np.eye(m)
            ctx.transform_gram(t, xs)  # warm
            ctx.gemm_inner(xs, xs)
            ctx.synchronize()
            ctx.ledger_reset()
            ctx.ledger_enable(True)
            for _ in range(a.reps):
                ctx.transform_gram(t, xs, gram=True)
                ctx.transform_gram(t, xs, gram=False)
                ctx.gemm_inner(xs, xs)
            ctx.synchronize()
            led = ctx.ledger()
            ctx.ledger_enable(False)
            row = {k: {"avg_us": round(1e3 * v["ms"] / v["calls"], 1), "GBs": round(v["bytes"] / v["ms"] / 1e6, 1)}
                   for k, v in led.items()}
            out[f"n={n} m={m}"] = row
            print(f"n={n} m={m}", json.dumps(row), flush=True)
            for x in xs:
                x.free()
print(json.dumps(out))
