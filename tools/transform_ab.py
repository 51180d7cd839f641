#!/usr/bin/env python3
"""k_transform with its Gram / self-dots (the block orthonormalisation's CholeskyQR2 passes): the
doubled window for m > 4 (SSP_TRANSFORM_WIDE=1, two waves per SIMD; the default for the self-dot instance since) against the narrow one, on the SAME
vectors: one context per setting (read at context creation), settings alternated call by call in one
process.  HIP-event ledger of each context, median over the rounds.

usage: python tools/transform_ab.py [--settings 0,1] [--rounds 9] [--out gpurun_out/transform_ab.json]
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
    ap.add_argument("--settings", default="0,1")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--ns", default="12500000,100000000")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "transform_ab.json"))
    a = ap.parse_args()
    settings = [int(v) for v in a.settings.split(",")]
    ctxs = {}
    for v in settings:
        os.environ["SSP_TRANSFORM_WIDE"] = str(v)
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
            row = {"n": n, "op": name, **{f"GBs_wide_{v}": round(nbytes / (float(np.median(t[v])) / 1e3) / 1e9, 1)
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
