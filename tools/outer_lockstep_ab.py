#!/usr/bin/env python3
"""A/B of gemm_outer's lockstep source groups (csrc/kernels_panel.hip, default) against free-running
waves (SSP_OUTER_LOCKSTEP=0), alternating processes so that placement and clocks affect both alike:
the read-modify-write 48 -> 8 (the bench's dominant kernel), the write-only 48 -> 8 (construct_solution),
64 -> 16 and 1 -> 8 at N = 1e8, library HIP-event ledger, median of 7.

usage: python tools/outer_lockstep_ab.py [--rounds 3] [--out gpurun_out/outer_lockstep_ab.json]

Result (profiles/r3/outer_lockstep_ab.json): no gain, so the lockstep form and its SSP_OUTER_LOCKSTEP
knob were removed from the library again; rerunning this tool needs that change re-applied.
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
n = 10**8
pool = [ctx.alloc(n) for _ in range(80)]
for i, v in enumerate(pool):
    ctx.fill_random(v, 7, i)
rng = np.random.default_rng(0)
out = {}
cases = {}
for k, m in ((48, 8), (64, 16), (1, 8)):
    al = rng.uniform(-1e-3, 1e-3, (k, m))
    cases[f"rmw {k}->{m}"] = (lambda al=al, k=k, m=m: ctx.gemm_outer(al, pool[16:16 + k], pool[:m]), 8.0 * n * (k + 2 * m))
al = rng.uniform(-1e-3, 1e-3, (48, 8))
cases["set 48->8"] = (lambda: ctx.gemm_outer_set(al, pool[16:64], pool[:8]), 8.0 * n * 56)
for name, (fn, nb) in cases.items():
    t = []
    for r in range(8):
        ctx.synchronize(); ctx.ledger_reset(); ctx.ledger_enable(True)
        fn()
        ctx.synchronize(); led = ctx.ledger(); ctx.ledger_enable(False)
        if r:
            t.append(sum(e["ms"] for e in led.values()))
    out[name] = nb / 1e6 / float(np.median(t))
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "outer_lockstep_ab.json"))
    a = ap.parse_args()
    res = {"lockstep": [], "free": []}
    for _ in range(a.rounds):
        for mode in ("free", "lockstep"):
            env = dict(os.environ, SSP_OUTER_LOCKSTEP="0" if mode == "free" else "1")
            p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "iterative-solver_amd")], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            res[mode].append(r)
            print(mode, json.dumps({k: round(v, 1) for k, v in r.items()}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
