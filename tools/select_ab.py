#!/usr/bin/env python3
"""k_select_local's workgroup merges, threshold-and-rank (default) against the LDS tree alone
(SSP_SELECT_MERGE=tree), on the SAME vectors: one context per setting (read at context creation),
settings alternated call by call in one process.  Checks that both give the same selection and
prints the HIP-event ledger's device time per call (median over the rounds).

usage: python tools/select_ab.py [--ns 1.5e5,1.25e7,1e8] [--nsel 8,16] [--rounds 9] [--out gpurun_out/select_ab.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402

SETTINGS = ("rank", "tree")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1.5e5,1.25e7,1e8")
    ap.add_argument("--nsel", default="8,16")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "select_ab.json"))
    a = ap.parse_args()
    ctxs = {}
    for v in SETTINGS:
        os.environ["SSP_SELECT_MERGE"] = v
        ctxs[v] = sh.Context(0)
    home = ctxs[SETTINGS[0]]
    res = []
    for n in (int(float(x)) for x in a.ns.split(",")):
        x = home.alloc(n)
        cases = (("uniform", lambda: home.fill_random(x, 1, 0), False),
                 ("diag_min", lambda: home.synthetic_diagonal(x, 0.1, 8), False),
                 ("diag_max", lambda: home.synthetic_diagonal(x, 0.1, 8), True))
        for name, fill, mx in cases:
            fill()
            home.synchronize()
            for nsel in (int(s) for s in a.nsel.split(",")):
                t = {v: [] for v in SETTINGS}
                got = {}
                for r in range(a.rounds + 1):
                    for v in SETTINGS:
                        c = ctxs[v]
                        c.ledger_reset()
                        c.ledger_enable(True)
                        idx, val = c.select(x, nsel, max=mx)
                        c.ledger_enable(False)
                        e = c.ledger()["select"]
                        got[v] = (idx.tolist(), val.tobytes())
                        if r:
                            t[v].append(1e3 * e["ms"] / e["calls"])
                same = got[SETTINGS[0]] == got[SETTINGS[1]]
                row = {"case": name, "n": n, "nsel": nsel, "same": same,
                       **{f"device_us_{v}": round(float(np.median(t[v])), 1) for v in SETTINGS}}
                print(json.dumps(row), flush=True)
                res.append(row)
                if not same:
                    raise SystemExit("select_ab: the two merges disagree")
        x.free()
        home.release_cached()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
