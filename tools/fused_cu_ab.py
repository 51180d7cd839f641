#!/usr/bin/env python3
"""The fused window passes (transform with its Gram / self-dots, axpy_pairs_norm, precondition_norms)
against their launch's workgroups per CU, on the SAME vectors: one context per setting
(SSP_FUSED_PER_CU is read at context creation), settings alternated call by call in one process (the
vectors' placement is common to all).  The default 8 per CU asks for more workgroups than these
kernels keep resident (4-6 per CU), so a second, partial round of workgroups runs at low occupancy.
HIP-event ledger of each context, median over the rounds.

usage: python tools/fused_cu_ab.py [--settings 8,4,6] [--rounds 7] [--out gpurun_out/fused_cu_ab.json]
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
    ap.add_argument("--settings", default="8,4,6")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--ns", default="12500000,100000000")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "fused_cu_ab.json"))
    a = ap.parse_args()
    settings = [int(v) for v in a.settings.split(",")]
    ctxs = {}
    for v in settings:
        os.environ["SSP_FUSED_PER_CU"] = str(v)
        ctxs[v] = sh.Context(0)
    home = ctxs[settings[0]]
    m = 8
    rng = np.random.default_rng(3)
    t8 = np.eye(m) + rng.uniform(-1e-3, 1e-3, (m, m))
    res = []
    for n in (int(float(x)) for x in a.ns.split(",")):
        xs = [home.alloc(n) for _ in range(m)]
        ys = [home.alloc(n) for _ in range(m)]
        d = home.alloc(n)
        for i, v in enumerate(xs + ys + [d]):
            home.fill_random(v, 5, i)
        home.synchronize()
        ops = {
            "transform_gram": ("transform_gram", lambda c: c.transform_gram(t8, xs)),
            "transform_norms": ("transform_gram", lambda c: c.transform_norms(t8, xs)),
            "axpy_pairs_norm": ("axpy_pairs_norm", lambda c: c.axpy_pairs_norm([1e-3] * m, ys, xs)),
            "precondition_norms": ("precondition", lambda c: c.precondition_norms(xs, d, [0.5] * m)),
        }
        for name, (ledger_op, call) in ops.items():
            t = {v: [] for v in settings}
            for r in range(a.rounds + 1):
                for v in settings:
                    c = ctxs[v]
                    c.ledger_reset()
                    c.ledger_enable(True)
                    call(c)
                    c.synchronize()
                    c.ledger_enable(False)
                    led = c.ledger()
                    if r:
                        t[v].append(sum(e["ms"] for e in led.values()))
                        nbytes = sum(e["bytes"] for e in led.values())
            row = {"n": n, "op": name, **{f"GBs_per_cu_{v}": round(nbytes / (float(np.median(t[v])) / 1e3) / 1e9, 1)
                                          for v in settings}}
            print(json.dumps(row), flush=True)
            res.append(row)
        for v in xs + ys + [d]:
            v.free()
        home.release_cached()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
