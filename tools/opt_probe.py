"""GPU vs independent restatement on the BFGS Rayleigh-quotient cases (development probe)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "iterative-solver_amd")]
import numpy as np  # noqa: E402

import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402
import test_davidson_independent as t  # noqa: E402

with sh.Context(0) as ctx:
    for mat, q in [("random60", 4), ("random60", 0), ("bh", 0), ("simplified", 4), ("he", 0)]:
        kw, ref, ind = t._run_opt(mat, "BFGS", q)
        gpu = ih.optimize_dense(ctx, t.OPT_M[mat], "BFGS", **kw)
        gpu["trace"] = {k: np.asarray(v).tolist() for k, v in gpu["trace"].items()}
        print(mat, q, "iterations gpu/cpu/np", gpu["iterations"], ref["iterations"], ind["iterations"],
              "first divergence gpu-np", t.first_divergence(gpu["trace"], ind["trace"]),
              "gpu-cpu", t.first_divergence(gpu["trace"], ref["trace"]), "conv", gpu["converged"], flush=True)
