#!/usr/bin/env python3
"""Does gemm_outer (48 -> 8 read-modify-write, N = 1e8) run slower inside the bench step than alone?
The bench's ledger puts it at 9.37 ms (5.46 TB/s, profiles/r3/bench_v4.json), the isolated A/B at
9.07 ms (5.64 TB/s, profiles/r3/outer_lockstep_ab.json).  The bench step precedes every gemm_outer
with fill(0) of its 8 destinations and two gemm_inner; this times the gemm_outer alone (library
HIP-event ledger, median of 7) after each preceding operation, in one process per round.

usage: python tools/outer_context_probe.py [--rounds 2] [--out gpurun_out/outer_context_probe.json]
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
m, k = 8, 48
rp = [ctx.alloc(n) for _ in range(m)]
ra = [ctx.alloc(n) for _ in range(m)]
qp = [ctx.alloc(n) for _ in range(k)]
qa = [ctx.alloc(n) for _ in range(k)]
for i, v in enumerate(rp + ra + qp + qa):
    ctx.fill_random(v, 7, i)
rng = np.random.default_rng(0)
coef = rng.uniform(-0.1, 0.1, (k, m))
def timed(fn):
    ctx.synchronize(); ctx.ledger_reset(); ctx.ledger_enable(True)
    fn()
    ctx.synchronize(); led = ctx.ledger(); ctx.ledger_enable(False)
    return sum(e["ms"] for e in led.values())
def run(pre, fn):
    t = []
    for r in range(8):
        pre()
        ms = timed(fn)
        if r:
            t.append(ms)
    return 8.0 * n * (k + 2 * m) / 1e6 / float(np.median(t))
outer = lambda: ctx.gemm_outer(coef, qp, rp)
def fill(val):
    def f():
        for v in rp:
            ctx.fill(val, v)
    return f
def inner():
    ctx.gemm_inner(rp, qp); ctx.gemm_inner(rp, qa)
def bench_order():
    inner(); fill(0.0)()
out = {
    "alone": run(lambda: None, outer),
    "after fill(0)": run(fill(0.0), outer),
    "after fill(1e-3)": run(fill(1e-3), outer),
    "after 2 gemm_inner": run(inner, outer),
    "after 2 gemm_inner + fill(0) (bench order)": run(bench_order, outer),
    "after fill_random": run(lambda: [ctx.fill_random(v, 9, i) for i, v in enumerate(rp)], outer),
}
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "outer_context_probe.json"))
    a = ap.parse_args()
    res = []
    for _ in range(a.rounds):
        p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "iterative-solver_amd")],
                           capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            print(p.stdout[-2000:], p.stderr[-3000:])
            sys.exit(p.returncode)
        r = json.loads(p.stdout.strip().splitlines()[-1])
        res.append(r)
        print(json.dumps({k: round(v, 1) for k, v in r.items()}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
