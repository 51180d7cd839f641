"""The north-star trace bar shared by the single-GPU trace tests (test_traces_gpu.py) and the sharded
ones (dist_worker.py gpu_traces): a solver run against a committed per-iteration trace of the
reference CPU path (tests/golden/traces.json, tests/golden/make_traces.py).  The bar itself is
described in test_traces_gpu.py's docstring."""
import json
import os

import numpy as np

T = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "traces.json")))
C5 = sorted(k for k, v in T.items() if not k.startswith("_") and k.startswith("C5_"))


def problem_kw(c):
    """The synthetic family of a trace case (diag_kind / alpha / target; absent = d_g = 1 + g and the
    solution x = 1), make_traces.py."""
    return {k: c[k] for k in ("diag_kind", "alpha", "target") if k in c}


def run_case(ih, ctx, ref, **kw):
    """The product solver (itsolv_hbm) on a trace case's problem and options."""
    c = ref["case"]
    run = ih.diis_synthetic if c["kind"] == "diis" else ih.davidson_synthetic
    return run(ctx, c["n"], c["rho"], c["rank"], c["seed"], **problem_kw(c), **kw, **ref["options"])
DAVIDSON = sorted(k for k, v in T.items() if not k.startswith("_") and v["case"]["kind"] == "davidson")
EIG_REL, ERR_REL, ERR_ABS, DEV_FACTOR = 1e-10, 1e-6, 1e-13, 10.0


# make_traces.py VARIANTS: valid sum orders of the CPU path -- a vectorising and a blocked build of its
# loops, and (where generated: the RS cases) the reference's distributed build on 2..16 MPI ranks with rank-order
# sums (one valid MPI_Allreduce association)
VARIANTS = ("reordered", "reordered_blocked", "mpi2", "mpi3", "mpi4", "mpi8", "mpi16")


def variants(ref):
    return [ref[k] for k in VARIANTS if k in ref]


def error_tolerance(ref):
    """Per-iteration absolute tolerance on the errors: ERR_REL * e + DEV_FACTOR * (the reference CPU
    path's own deviation under its reordered sums, max over the variants, the iteration and its two
    neighbours)."""
    e = np.array(ref["trace"]["errors"])
    dev = np.zeros(len(e))
    for v in variants(ref):
        d = np.array(v["error_abs_dev"][:len(e)])
        dev[:len(d)] = np.maximum(dev[:len(d)], d)
    win = np.maximum.reduce([dev, np.r_[dev[1:], 0.0], np.r_[0.0, dev[:-1]]])
    return ERR_REL * e + DEV_FACTOR * win[:, None] + ERR_ABS


def same_steps(ref):
    """True where every reordered CPU path takes the reference's steps (the strict step bar applies)."""
    return all(v["same_steps"] for v in variants(ref))


def assert_trace(gpu, ref, name):
    assert gpu["converged"] == ref["converged"], name
    assert gpu["iterations"] == ref["iterations"], (name, gpu["iterations"], ref["iterations"])
    g, r = gpu["trace"], ref["trace"]
    if same_steps(ref):
        assert gpu["r_creations"] == ref["r_creations"], (name, gpu["r_creations"], ref["r_creations"])
        assert gpu["q_creations"] == ref["q_creations"], name
        assert list(g["nq"]) == r["nq"], (name, list(g["nq"]), r["nq"])
        assert list(g["nwork"]) == r["nwork"], name
        if "screened" in r:  # propose_rspace's redundancy / null screening, iteration by iteration
            assert list(g["screened"]) == r["screened"], (name, list(g["screened"]), r["screened"])
            assert (gpu["redundant_params"], gpu["null_params"]) == (ref["redundant_params"], ref["null_params"]), name
    if r["eigenvalues"]:
        re = np.array(r["eigenvalues"])
        de = np.abs(g["eigenvalues"] - re)
        assert np.all(de <= EIG_REL * np.maximum(np.abs(re), 1.0)), (name, de.max())
    rr = np.array(r["errors"])
    dr = np.abs(g["errors"] - rr)
    tol = error_tolerance(ref)
    q = dr / tol
    worst = np.unravel_index(np.argmax(q), q.shape)
    assert np.all(dr <= tol), (name, "iteration", int(worst[0]), "error", float(rr[worst]), "deviation",
                               float(dr[worst]), "tolerance", float(tol[worst]), "ratio", float(q[worst]))
    # the reported run ends where the reference's does: converged errors below the threshold
    if ref["converged"]:
        assert np.max(g["errors"][-1]) <= ref["options"]["convergence_threshold"], name


def solution_target(ref):
    """The component value of a nonlinear-equations trace case's solution (r = H (x - target 1))."""
    return ref["case"].get("target", 1.0)
