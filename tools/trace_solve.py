#!/usr/bin/env python3
"""Two solves of a solver_ledger config with the ledger OFF (no event records between ops), for a
kernel / HIP-API trace of the production path (development tool).
usage: python tools/trace_solve.py [--config C4-shard]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402
from solver_ledger import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4-shard")
a = ap.parse_args()
solver, n, kw = CONFIGS[a.config]
kw = dict(kw)
rho, rank, seed = kw.pop("rho"), kw.pop("rank"), kw.pop("seed")
with sh.Context(0) as ctx:
    for i in range(2):
        t0 = time.perf_counter()
        if solver == "davidson":
            r = ih.davidson_synthetic(ctx, n, rho, rank, seed, n_local=0, **kw)
        else:
            r = ih.diis_synthetic(ctx, n, rho, rank, seed, n_local=0, **kw)
        print(a.config, "solve", i, "wall_ms", round(1e3 * (time.perf_counter() - t0), 2), "iterations", r["iterations"],
              flush=True)
        time.sleep(0.05)  # a clear gap between the solves in the trace
