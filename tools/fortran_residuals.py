"""Per-case outcomes of the Fortran callers (tests/fortran_cases.py run_all) on the HIP path, for A/B
runs of a host-side choice (e.g. SSP_ORTHO=two_pass): iterations and residual of every linear-equation
case, iterations of every eigen case.  GPU only; writes JSON.

usage: python tools/fortran_residuals.py OUT.json [--lineq] [--emul] [SEED ...]   (--emul: the CPU path)   (seeds: fortran_cases.perturb; default 0)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import fortran_cases as fc  # noqa: E402


def run_lineq(lib, seed):
    """The linear-equation cases of fortran_cases.run_all alone."""
    import numpy as np
    res = {}
    for n in range(3, 34, 3):
        for nroot in range(1, min(n, 13) + 1):
            m, rhs = fc.lineq_problem(n, nroot)
            m = np.asfortranarray(fc.perturb(m, seed))
            rhs = np.asfortranarray(fc.perturb(rhs, seed + 50 if 0 < seed < 100 else seed))
            sol, rn = np.zeros((n, nroot), order="F"), np.zeros(1)
            it = lib.f_linear_equations(fc._p(m), fc._p(rhs), n, nroot, 0.0, 1e-10, fc._p(sol), fc._p(rn))
            res[f"lineq/{n}/{nroot}"] = {"iterations": it, "residual": float(rn[0])}
    return res


def main():
    lib = fc.load(fc.LIB_EMUL if "--emul" in sys.argv else fc.LIB_GPU)
    lineq_only = "--lineq" in sys.argv
    seeds = [int(s) for s in sys.argv[2:] if not s.startswith("--")] or [0]
    runs = {}
    for seed in seeds:
        res = run_lineq(lib, seed) if lineq_only else fc.run_all(lib, seed)
        out = {k: {"iterations": v.get("iterations"), "residual": v.get("residual")} for k, v in res.items()
               if k.startswith(("lineq/", "eigen/"))}
        runs[str(seed)] = out
        worst = sorted((v["residual"], k) for k, v in out.items() if v["residual"] is not None)[-3:]
        print("seed", seed, "worst lineq residuals:", worst, flush=True)
    with open(sys.argv[1], "w") as f:
        json.dump({"ortho": os.environ.get("SSP_ORTHO", "one_pass"), "runs": runs}, f, indent=0)


if __name__ == "__main__":
    main()
