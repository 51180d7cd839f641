#!/usr/bin/env python3
"""A/B of the gemm_inner row kernel's two shapes (csrc/kernels_panel.hip): the window shape
(default) against round 2's grid-stride shape (SSP_ROW_SHAPE=stride), alternating processes so that
placement and clocks affect both alike.  Per process: 1 x 1 (x.y and the norm x.x) and 1 x 2 panels
at N = 1e8 and at C4's shard N = 1.25e7 (library HIP-event ledger), and the DIIS runs whose
iteration counts depend on the summation order: C5 (tests/golden/traces.json C5_n1e7, 27 steps on the
CPU path) and the ill-conditioned case of tests/test_solver_gpu.py (n = 1e5, rank 2, rho 0.01).

usage: python tools/row_shape_ab.py [--rounds 2] [--out gpurun_out/row_shape_ab.json]
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
import subspace_hip as sh, itsolv_hbm as ih
ctx = sh.Context(0)
out = {"shapes": {}, "diis": {}}
for n in (10**8, 12_500_000):
    v = [ctx.alloc(n) for _ in range(3)]
    for i, x in enumerate(v):
        ctx.fill_random(x, 5, i)
    cases = {"1x1 x.y": (lambda: ctx.gemm_inner(v[:1], v[1:2]), 16.0 * n),
             "1x1 x.x": (lambda: ctx.gemm_inner(v[:1], v[:1]), 8.0 * n),
             "1x2": (lambda: ctx.gemm_inner(v[:1], v[1:3]), 24.0 * n)}
    for name, (fn, nb) in cases.items():
        t = []
        for r in range(9):
            ctx.synchronize(); ctx.ledger_reset(); ctx.ledger_enable(True)
            fn()
            ctx.synchronize(); led = ctx.ledger(); ctx.ledger_enable(False)
            if r:
                t.append(sum(e["ms"] for e in led.values()))
        out["shapes"][f"{name} n={n}"] = nb / 1e6 / float(np.median(t))
    for x in v:
        x.free()
c5 = ih.c5_spec(10_000_000)
r = ih.diis_synthetic(ctx, 10_000_000, solutions=False, max_size_qspace=6, convergence_threshold=1e-8, **c5)
out["diis"]["C5 n=1e7"] = r["iterations"]
r = ih.diis_synthetic(ctx, 100_000, 0.01, 2, 3, solutions=False, max_size_qspace=6, convergence_threshold=1e-8)
out["diis"]["n=1e5 rank 2 rho 0.01"] = r["iterations"]
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "row_shape_ab.json"))
    a = ap.parse_args()
    res = {"window": [], "stride": []}
    for _ in range(a.rounds):
        for shape in ("stride", "window"):
            env = dict(os.environ)
            env.pop("SSP_ROW_SHAPE", None)
            if shape == "stride":
                env["SSP_ROW_SHAPE"] = "stride"
            p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "iterative-solver_amd")], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            res[shape].append(r)
            print(shape, json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
