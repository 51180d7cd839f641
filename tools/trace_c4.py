#!/usr/bin/env python3
"""Runs the C4-shard Davidson solve (C3's problem at N = 1.25e7, one rank's share of C4) a few times
with the op ledger OFF, for a kernel trace whose gaps are the solve's own idle (the ledger's HIP
events add host work between ops).  Prints each solve's wall time and host-algebra time.

usage: rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/trace_c4.py [--n N] [--repeat R]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))

import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402

C3 = dict(rho=0.1, rank=8, seed=1, nroots=8, max_p=16, max_size_qspace=48, reset_D=8, convergence_threshold=1e-8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12_500_000)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    ctx = sh.Context(0)
    for rep in range(a.repeat):
        t0 = time.perf_counter()
        r = ih.davidson_synthetic(ctx, a.n, n_local=0, solutions=False, **C3)
        ctx.synchronize()
        wall = time.perf_counter() - t0
        print(json.dumps({"tag": a.tag, "rep": rep, "wall_ms": round(1e3 * wall, 3), "iterations": r["iterations"],
                          "host_algebra_ms": round(1e3 * r["host_algebra"]["seconds"], 3),
                          "host_algebra_calls": r["host_algebra"]["calls"]}), flush=True)
        time.sleep(0.01)  # a marker gap between solves in the trace
    ctx.close()


if __name__ == "__main__":
    main()
