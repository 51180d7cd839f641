#!/usr/bin/env python3
"""Times ssp_select on one shard for a few input distributions and selection sizes: wall time per
call and the HIP-event ledger's device time (kernel-level detail: run under rocprofv3 --kernel-trace
--stats).  Development probe.

usage: python tools/select_probe.py [N] [--nsel 8,16,1024]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=float, default=1e8)
    ap.add_argument("--nsel", default="8,16,1024")
    a = ap.parse_args()
    n = int(a.n)
    with sh.Context(0) as ctx:
        x = ctx.alloc(n)
        cases = (("uniform", lambda: ctx.fill_random(x, 1, 0), False),
                 ("diag_min", lambda: ctx.synthetic_diagonal(x, 0.1, 8), False),
                 ("diag_max", lambda: ctx.synthetic_diagonal(x, 0.1, 8), True))
        for name, fill, mx in cases:
            fill()
            ctx.synchronize()
            for nsel in (int(s) for s in a.nsel.split(",")):
                ctx.select(x, nsel, max=mx)
                ctx.ledger_reset()
                ctx.ledger_enable(True)
                t0 = time.perf_counter()
                for _ in range(5):
                    ctx.select(x, nsel, max=mx)
                dt = (time.perf_counter() - t0) / 5
                ctx.ledger_enable(False)
                e = ctx.ledger().get("select", {"ms": 0.0, "calls": 1})
                print(json.dumps({"case": name, "n": n, "nsel": nsel, "wall_us": round(dt * 1e6, 1),
                                  "device_us": round(1e3 * e["ms"] / max(1, e["calls"]), 1)}), flush=True)


if __name__ == "__main__":
    main()
