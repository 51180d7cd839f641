#!/usr/bin/env python3
"""Times ssp_select on one shard of N = 1e8 for a few input distributions (kernel-level detail:
run under rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
with sh.Context(0) as ctx:
    x = ctx.alloc(n)
    for name, fill in (("uniform", lambda: ctx.fill_random(x, 1, 0)),
                       ("diag", lambda: ctx.synthetic_diagonal(x, 0.1, 8))):
        fill()
        ctx.synchronize()
        for nsel in (16, 1024):
            ctx.select(x, nsel)
            t0 = time.perf_counter()
            for _ in range(5):
                ctx.select(x, nsel)
            dt = (time.perf_counter() - t0) / 5
            print(f"{name:8s} nsel={nsel:5d} {dt * 1e6:9.1f} us  {8 * n / dt / 1e9:7.1f} GB/s", flush=True)
