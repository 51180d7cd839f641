#!/usr/bin/env python3
"""gemm_outer 48 -> 8 at N = 1e8 over several independently allocated vector sets in ONE process
(the placement spread of DESIGN.md §4): per set, 3 calls timed by the library's HIP-event ledger.
Run under rocprofv3 --pmc to correlate a set's rate with per-dispatch counters (dispatch order:
set 0 calls 0..2, set 1 calls 0..2, ...).

usage: python tools/outer_placement_probe.py [--sets 4] [--out gpurun_out/outer_placement_probe.json]
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
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "outer_placement_probe.json"))
    a = ap.parse_args()
    n, m, k = int(a.n), 8, 48
    ctx = sh.Context(0)
    coef = np.random.default_rng(0).uniform(-0.1, 0.1, (k, m))
    sets = []
    for s in range(a.sets):
        rp = [ctx.alloc(n) for _ in range(m)]
        qp = [ctx.alloc(n) for _ in range(k)]
        for i, v in enumerate(rp + qp):
            ctx.fill_random(v, 7, i)
        sets.append((rp, qp))
    ctx.synchronize()
    res = []
    for s, (rp, qp) in enumerate(sets):
        rates = []
        for _ in range(3):
            ctx.ledger_reset()
            ctx.ledger_enable(True)
            ctx.gemm_outer(coef, qp, rp)
            ctx.synchronize()
            led = ctx.ledger()
            ctx.ledger_enable(False)
            rates.append(8.0 * n * (k + 2 * m) / 1e6 / sum(e["ms"] for e in led.values()))
        ptrs = [hex(int(getattr(v.ptr, "value", v.ptr) or 0)) for v in rp + qp][:3]
        res.append({"set": s, "GBs": rates, "first_ptrs": ptrs})
        print(s, [round(r) for r in rates], flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
