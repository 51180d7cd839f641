#!/usr/bin/env python3
"""Whole-solve wall times with the ledger off (development tool), for A/Bs of host-side knobs that
act between kernels (environment variables read at context creation): one process runs the
C4-shard Davidson solve (tools/solver_ledger.py's C4-shard) `--repeat` times after one cold solve
and prints one JSON line with every warm wall time, their median and minimum.

usage: python tools/wall_ab.py [--config C4-shard] [--repeat 8] [--tag NAME]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402
from solver_ledger import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4-shard")
    ap.add_argument("--repeat", type=int, default=8)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    solver, n, kw = CONFIGS[a.config]
    kw = dict(kw)
    rho, rank, seed = kw.pop("rho"), kw.pop("rank"), kw.pop("seed")
    ctx = sh.Context(0)
    walls, its, ev = [], None, None
    for rep in range(a.repeat + 1):
        t0 = time.perf_counter()
        if solver == "davidson":
            r = ih.davidson_synthetic(ctx, n, rho, rank, seed, n_local=0, **kw)
        else:
            r = ih.diis_synthetic(ctx, n, rho, rank, seed, n_local=0, **kw)
        ctx.synchronize()
        w = time.perf_counter() - t0
        its = r["iterations"]
        ev = [float(e).hex() for e in r.get("eigenvalues", [])][:8] if solver == "davidson" else None
        if rep:
            walls.append(w)
    ctx.close()
    print(json.dumps({"tag": a.tag, "config": a.config, "iterations": its, "eigenvalues_hex": ev,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("SSP_")},
                      "wall_ms": [round(1e3 * w, 3) for w in walls],
                      "median_ms": round(1e3 * statistics.median(walls), 3),
                      "min_ms": round(1e3 * min(walls), 3)}), flush=True)


if __name__ == "__main__":
    main()
