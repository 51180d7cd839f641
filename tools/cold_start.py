#!/usr/bin/env python3
"""Where does the first solve in a process go?  (C2 cold 4.47 s vs 0.074 s warm.)

Each phase runs in a FRESH process (so code objects, HIP runtime state and the HBM arena start cold):
  plain     ctx create, C2 solve (cold), C2 solve (warm)
  kernels   ctx create, every kernel once at n = 4096 (code-object load), C2 solve
  alloc     ctx create, the C2 solve's HBM blocks allocated + freed once (arena warm), C2 solve
  touch     as alloc, plus one fill of every block before freeing (first-touch of the pages)
usage: python tools/cold_start.py [--out gpurun_out/cold_start.json] [--n 1e7]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))

C2 = dict(rho=0.1, rank=8, seed=1, nroots=4, max_size_qspace=24, reset_D=8, convergence_threshold=1e-8)
NBLOCKS = 64  # > the 2 (nQ + nroots) + P + D + workspace vectors a C2 solve holds


def phase(name, n):
    t0 = time.perf_counter()
    import itsolv_hbm as ih
    import subspace_hip as sh

    ih.load_library()
    t_import = time.perf_counter() - t0
    t0 = time.perf_counter()
    ctx = sh.Context(0)
    ctx.synchronize()
    out = {"phase": name, "n": n, "import_s": round(t_import, 3), "ctx_create_s": round(time.perf_counter() - t0, 3)}
    if name == "kernels":
        t0 = time.perf_counter()
        small = 4096
        a = [ctx.alloc(small) for _ in range(8)]
        for v in a:
            ctx.fill(1.0, v)
        ctx.scal(2.0, a[0])
        ctx.copy(a[1], a[0])
        ctx.axpy(0.5, a[0], a[1])
        ctx.dot(a[0], a[1])
        ctx.dot(a[0], a[0])
        ctx.gemm_inner(a[:2], a[2:8])
        ctx.gemm_inner(a[:1], a[2:4])
        import numpy as np

        ctx.gemm_outer(np.ones((6, 2)), a[2:8], a[:2])
        ctx.synchronize()
        out["kernel_warmup_s"] = round(time.perf_counter() - t0, 3)
    if name in ("alloc", "touch"):
        t0 = time.perf_counter()
        blocks = [ctx.alloc(n) for _ in range(NBLOCKS)]
        out["alloc_s"] = round(time.perf_counter() - t0, 3)
        if name == "touch":
            t0 = time.perf_counter()
            for b in blocks:
                ctx.fill(0.0, b)
            ctx.synchronize()
            out["first_touch_s"] = round(time.perf_counter() - t0, 3)
        del blocks
        ctx.synchronize()
    t0 = time.perf_counter()
    r = ih.davidson_synthetic(ctx, n, n_local=0, **C2)
    out["solve1_s"] = round(time.perf_counter() - t0, 3)
    out["solve1_inner_s"] = round(r["seconds"], 3)
    t0 = time.perf_counter()
    r2 = ih.davidson_synthetic(ctx, n, n_local=0, **C2)
    out["solve2_s"] = round(time.perf_counter() - t0, 3)
    out["iterations"] = [r["iterations"], r2["iterations"]]
    ctx.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--phase")
    ap.add_argument("--n", type=float, default=1e7)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cold_start.json"))
    a = ap.parse_args()
    if a.phase:
        phase(a.phase, int(a.n))
        return
    res = []
    for p in ("plain", "kernels", "alloc", "touch", "plain"):
        t0 = time.perf_counter()
        r = subprocess.run([sys.executable, __file__, "--phase", p, "--n", str(a.n)], capture_output=True, text=True,
                           timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        d = json.loads(line[-1]) if line else {"phase": p, "error": r.stderr[-2000:]}
        d["process_wall_s"] = round(time.perf_counter() - t0, 3)
        print(json.dumps(d), flush=True)
        res.append(d)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
