#!/usr/bin/env python3
"""Host-buffer boundary rate: what the reference's C / Fortran / Python API path (R vectors in host
memory, uploaded before and downloaded after every solver call; host/iterative_solver_c.cpp upload /
download) adds to the HBM-resident path.  Times ssp_upload / ssp_download of pageable numpy vectors
of N = 1e7 and 1e8 doubles and prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402

out = {}
with sh.Context(0) as ctx:
    for n in (10_000_000, 100_000_000):
        a = np.random.default_rng(1).uniform(-1, 1, n)
        v = ctx.upload(a)
        b = np.empty_like(a)
        ctx.upload_into(v, a)
        ctx.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.upload_into(v, a)
        ctx.synchronize()
        h2d = 8 * n * reps / (time.perf_counter() - t0) / 1e9
        t0 = time.perf_counter()
        for _ in range(reps):
            b = ctx.download(v)
        d2h_new = 8 * n * reps / (time.perf_counter() - t0) / 1e9
        # into the same (already touched) host array, as the C API writes the caller's R arrays
        t0 = time.perf_counter()
        for _ in range(reps):
            sh._check(ctx.lib.ssp_download(ctx.handle, b.ctypes.data, v.ptr, n))
        d2h = 8 * n * reps / (time.perf_counter() - t0) / 1e9
        assert np.array_equal(a, b)
        v.free()
        out[str(n)] = {"h2d_GBs": round(h2d, 2), "d2h_GBs": round(d2h, 2), "d2h_fresh_array_GBs": round(d2h_new, 2)}
print(json.dumps(out), flush=True)
