#!/usr/bin/env python3
"""gemm_outer_set 48 -> 8 and gemm_outer 48 -> 8 (read-modify-write) against the launch's workgroups per
CU, on the SAME vectors: one context per setting (SSP_OUTER_WG_PER_CU is read at context creation),
the settings alternated call by call in one process, so the vectors' physical placement -- which
decided more than the grid in round 3's one-process-per-setting A/B -- is common to all of them.
HIP-event ledger of each context, median over the rounds.

usage: python tools/outer_cu_ab.py [--settings 8,4,2] [--rounds 7] [--out gpurun_out/outer_cu_ab.json]
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
    ap.add_argument("--settings", default="8,4,2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--ns", default="12500000,100000000")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "outer_cu_ab.json"))
    a = ap.parse_args()
    settings = [int(v) for v in a.settings.split(",")]
    ctxs = {}
    for v in settings:
        os.environ["SSP_OUTER_WG_PER_CU"] = str(v)
        ctxs[v] = sh.Context(0)
    home = ctxs[settings[0]]
    m, k = 8, 48
    res = []
    for n in (int(float(x)) for x in a.ns.split(",")):
        rp = [home.alloc(n) for _ in range(m)]
        qp = [home.alloc(n) for _ in range(k)]
        for i, v in enumerate(rp + qp):
            home.fill_random(v, 7, i)
        home.synchronize()
        coef = np.random.default_rng(0).uniform(-0.1, 0.1, (k, m)) / k
        for op in ("gemm_outer_set", "gemm_outer"):
            t = {v: [] for v in settings}
            for r in range(a.rounds + 1):
                for v in settings:
                    c = ctxs[v]
                    c.ledger_reset()
                    c.ledger_enable(True)
                    getattr(c, op)(coef, qp, rp)
                    c.synchronize()
                    c.ledger_enable(False)
                    if r:
                        t[v].append(c.ledger()[op]["ms"])
            nbytes = 8.0 * n * (k + (m if op == "gemm_outer_set" else 2 * m))
            row = {"n": n, "op": op, **{f"GBs_per_cu_{v}": round(nbytes / (float(np.median(t[v])) / 1e3) / 1e9, 1)
                                         for v in settings}}
            print(json.dumps(row), flush=True)
            res.append(row)
        for v in rp + qp:
            v.free()
        home.release_cached()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
