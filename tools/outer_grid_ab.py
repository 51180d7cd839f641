#!/usr/bin/env python3
"""gemm_outer 48 -> 8 (read-modify-write) rate against the launch's workgroups per CU
(SSP_OUTER_WG_PER_CU), at the one-GPU size (N = 1e8) and the 8-GPU shard size (N = 1.25e7): one
process per (setting, round), settings alternated, library HIP-event ledger, median of 7 calls.

usage: python tools/outer_grid_ab.py [--rounds 2] [--settings 2,4,8,16] [--out gpurun_out/outer_grid_ab.json]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import subspace_hip as sh
ctx = sh.Context(0)
m, k = 8, 48
out = {}
for n in (12_500_000, 100_000_000):
    rp = [ctx.alloc(n) for _ in range(m)]
    qp = [ctx.alloc(n) for _ in range(k)]
    for i, v in enumerate(rp + qp):
        ctx.fill_random(v, 7, i)
    coef = np.random.default_rng(0).uniform(-0.1, 0.1, (k, m))
    t = []
    for r in range(8):
        ctx.synchronize(); ctx.ledger_reset(); ctx.ledger_enable(True)
        ctx.gemm_outer(coef, qp, rp)
        ctx.synchronize(); led = ctx.ledger(); ctx.ledger_enable(False)
        if r:
            t.append(sum(e["ms"] for e in led.values()))
    out[str(n)] = 8.0 * n * (k + 2 * m) / 1e6 / float(np.median(t))
    for v in rp + qp:
        v.free()
    ctx.release_cached()
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--settings", default="2,4,8,16")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "outer_grid_ab.json"))
    a = ap.parse_args()
    res = {s: [] for s in a.settings.split(",")}
    for _ in range(a.rounds):
        for s in res:
            env = dict(os.environ, SSP_OUTER_WG_PER_CU=s)
            p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "iterative-solver_amd")],
                               capture_output=True, text=True, timeout=600, env=env)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            res[s].append(r)
            print(s, json.dumps({kk: round(v, 1) for kk, v in r.items()}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
