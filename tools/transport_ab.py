#!/usr/bin/env python3
"""A/B of the rank transports on one MI355X (development tool): the same solve through a context with
no communicator (fused single-rank reductions), a one-rank RCCL communicator (fold -> ncclAllReduce
-> publish) and a one-rank peer-memory communicator (fold -> k_p2p_allreduce: push, flag wait,
rank-order sum, host publish), alternating in one process so that box and placement are shared.
Reports per transport the median wall time, kernel time (HIP-event ledger) and their difference.

usage: python tools/transport_ab.py [--config C4-shard] [--reps 5] [--out file.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402
from solver_ledger import CONFIGS, REDUCING  # noqa: E402


def solve(ctx, name, ledger):
    """One solve; with ledger=False the wall time carries no HIP-event records (each op's two
    hipEventRecord calls are host work on the path between a reduction and the next launch)."""
    solver, n, kw = CONFIGS[name]
    kw = dict(kw)
    rho, rank, seed = kw.pop("rho"), kw.pop("rank"), kw.pop("seed")
    ctx.ledger_reset()
    ctx.ledger_enable(ledger)
    ctx.synchronize()
    t0 = time.perf_counter()
    fn = ih.davidson_synthetic if solver == "davidson" else ih.diis_synthetic
    r = fn(ctx, n, rho, rank, seed, n_local=0, solutions=False, **kw)
    ctx.synchronize()
    wall = time.perf_counter() - t0
    ctx.ledger_enable(False)
    led = ctx.ledger()
    ms = sum(v["ms"] for v in led.values())
    red = sum(v["calls"] for op, v in led.items() if op.split("(")[0] in REDUCING)
    return {"wall_ms": 1e3 * wall, "kernel_ms": ms, "iterations": r["iterations"], "reductions": red}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4-shard")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ctxs = {"none": sh.Context(0), "rccl": sh.Context(0), "p2p": sh.Context(0)}
    ctxs["rccl"].attach_comm(1, 0, sh.Context.unique_id())
    ctxs["p2p"].attach_p2p(1, 0, sh.Context.p2p_unique_id())
    runs = {k: [] for k in ctxs}
    led = {k: [] for k in ctxs}
    for k, c in ctxs.items():  # warm: arena and code objects
        solve(c, a.config, True)
    for rep in range(a.reps):
        for k, c in ctxs.items():
            runs[k].append(solve(c, a.config, False))
            led[k].append(solve(c, a.config, True))
    out = {"config": a.config, "reps": a.reps,
           "note": "wall: ledger-off solves; kernel: HIP-event ledger of ledger-on solves of the same problem"}
    for k, rs in runs.items():
        wall = statistics.median(r["wall_ms"] for r in rs)
        wall_led = statistics.median(r["wall_ms"] for r in led[k])
        kern = statistics.median(r["kernel_ms"] for r in led[k])
        red = led[k][0]["reductions"]
        out[k] = {"wall_ms": round(wall, 2), "wall_ms_ledger_on": round(wall_led, 2), "kernel_ms": round(kern, 2),
                  "idle_ms": round(wall - kern, 2), "idle_frac_of_wall": round((wall - kern) / wall, 4),
                  "wall_ms_all": [round(r["wall_ms"], 2) for r in rs],
                  "iterations": rs[0]["iterations"], "reductions": red,
                  "idle_us_per_reduction": round(1e3 * (wall - kern) / max(1, red), 1)}
        print(k, json.dumps(out[k]), flush=True)
    for c in ctxs.values():
        c.close()
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
