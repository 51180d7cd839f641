"""Generates tests/golden/traces.json — per-iteration traces of the reference CPU path at the BASELINE
configurations, the fixtures the GPU solver must reproduce step for step (tests/test_traces_gpu.py).

The CPU path is the oracle: the restated solver stack over the restated ArrayHandlerIterable
(sequential std::inner_product / std::transform loops and pairwise gemm_*_default,
oracle/oracle_ops.c, built with -ffp-contract=off), i.e. the reference's CPU algorithm.  Each trace
records what the reference's driver exposes as parity observables (IterativeSolverTemplate.h:322-408,
LinearEigensystemDavidson.h:79): the iteration count, R/Q creations, convergence, and after every
iteration the eigenvalues and errors of every root, the Q-space size and the working-set size.
Each case is also run with the CPU path's dots summed in other valid orders ("reordered": 8
interleaved partial sums, what a vectorising build of the same loops does; "reordered_blocked":
1024-element blocks folded pairwise, what a blocked or threaded build does): that measures the
reference algorithm's own sensitivity to rounding, which is what a GPU (whose reductions also sum in
another order) can be held to -- same steps where every reordered CPU path takes the same steps, and
per-iteration errors within a few times the reordered CPU paths' own deviation.

Problem: H = diag(1 + i) + rho * sum_{l<rank} u_l u_l^T (rank 1 with u = 1 is the
reference's test_rayleigh_quotient.cpp:37-42 matrix at large n), options of §8d
(convergence_threshold 1e-8, max_size_qspace 6 * nroots, reset_D 8, max_p 16 for C3).

  C1  Davidson  1 root              N = 1e4   (rank 1 and rank 8)
  C2  Davidson  4 roots             N = 1e7   (rank 1 and the rank-8 perf problem)
  C3  Davidson  8 roots + P 16      N = 1e7   (C3's shape at a tenth of its length: the CPU path
                                               at N = 1e8 needs > 64 GB with 112 vectors)
  C3  Davidson  8 roots + P 16      N = 1e8   rank 1 (Q stays small: fits this container) and rank 8 (the
                                               bench's solve and C4's problem; Q grows to 48: ~100 GB,
                                               generated with --omp on a host with the memory)
  C5  DIIS      max_size_qspace 6   N = 1e7 and N = 1e8: the well-posed instance
                                              (itsolv_hbm/problems.h c5_spec: the reference test's
                                              1 1^T + diag form with the coupling scaled by 1/N, a
                                              bounded diagonal, a preconditioner diagonal mismatched
                                              by up to 20 % and the unit-norm solution 1/sqrt(N);
                                              |r_0| = 3.2, 10 steps to the 1e-8 threshold, the last
                                              two errors 2.8x above / 1.5x below it)
  RS  Davidson  8 roots (+ P 16)   N = 2^21  the redundancy screen's cases (propose_rspace.h:481-512):
                                              H = diag(1 + g) + rho 1 1^T, whose preconditioned residuals
                                              (D - lambda)^-1 r all lie close to the span of earlier
                                              (D - mu)^-1 1, so new R vectors are near-dependent and the
                                              screen removes 6 (P 16, rho 0.1) and 3 (rho 1) of them; above
                                              the fused-pass threshold (2^20), so the product runs its
                                              one-pass orthonormalisation and batched overlap rows on them
  C5x DIIS      max_size_qspace 6   N = 1e7   the round-1 instance (diag(1+g), rank 3, rho 0.01):
                                              |r_0| = 1.9e10, so the threshold lies below its rounding
                                              floor and the count past the 1e-6 plateau is decided by
                                              rounding (kept as the documented chaotic case: the
                                              12-iteration descent, threshold 1e-14, and the run)

Run (about 10 minutes on 8 cores, < 48 GB):  python tests/golden/make_traces.py [--only NAME ...]
C3_n1e8_rank8 (~100 GB):  ORACLE threads via OMP_NUM_THREADS; python tests/golden/make_traces.py --omp --only C3_n1e8_rank8
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "iterative-solver_amd"), os.path.join(ROOT, "oracle")]

RHO, SEED = 0.1, 1

CASES = {
    "C1_rank1": dict(kind="davidson", n=10_000, rho=RHO, rank=1, seed=SEED, nroots=1, max_p=0),
    "C1_rank8": dict(kind="davidson", n=10_000, rho=RHO, rank=8, seed=SEED, nroots=1, max_p=0),
    "C2_rank1": dict(kind="davidson", n=10_000_000, rho=RHO, rank=1, seed=SEED, nroots=4, max_p=0),
    "C2_rank8": dict(kind="davidson", n=10_000_000, rho=RHO, rank=8, seed=SEED, nroots=4, max_p=0),
    "C3_n1e7_rank1": dict(kind="davidson", n=10_000_000, rho=RHO, rank=1, seed=SEED, nroots=8, max_p=16),
    "C3_n1e7_rank8": dict(kind="davidson", n=10_000_000, rho=RHO, rank=8, seed=SEED, nroots=8, max_p=16),
    "C3_n1e8_rank1": dict(kind="davidson", n=100_000_000, rho=RHO, rank=1, seed=SEED, nroots=8, max_p=16),
    # the bench's own solve (bench.py in_solver) and C4's problem at full size: ~100 GB, run on a host
    # with the memory (--omp, the bit-identical OpenMP build of the CPU path)
    "C3_n1e8_rank8": dict(kind="davidson", n=100_000_000, rho=RHO, rank=8, seed=SEED, nroots=8, max_p=16),
    # C5: the well-posed DIIS instance (itsolv_hbm.c5_spec)
    "C5_n1e7": dict(kind="diis", n=10_000_000, rho=1.0 / 10_000_000, rank=1, seed=3, diag_kind=1, alpha=0.2,
                    target=10_000_000 ** -0.5, convergence_threshold=1e-8),
    "C5_n1e8": dict(kind="diis", n=100_000_000, rho=1.0 / 100_000_000, rank=1, seed=3, diag_kind=1, alpha=0.2,
                    target=100_000_000 ** -0.5, convergence_threshold=1e-8),
    # RS: near-dependent R vectors at 2^21 elements (the redundancy screen fires; fused passes on)
    "RS_n2e21_p16": dict(kind="davidson", n=2 ** 21, rho=0.1, rank=1, seed=SEED, nroots=8, max_p=16),
    "RS_n2e21_rho1": dict(kind="davidson", n=2 ** 21, rho=1.0, rank=1, seed=SEED, nroots=8, max_p=0),
    # C5x: the round-1 DIIS problem (profiles/r1/solver_ledger_v10.json: rho 0.01, rank 3, seed 3), chaotic
    "C5x_n1e7_traj12": dict(kind="diis", n=10_000_000, rho=0.01, rank=3, seed=3, max_iter=12,
                            convergence_threshold=1e-14),
    "C5x_n1e7": dict(kind="diis", n=10_000_000, rho=0.01, rank=3, seed=3, convergence_threshold=1e-8),
}


def problem_kw(c):
    """The synthetic family of a case (diag_kind / alpha; absent = the Davidson family d_g = 1 + g)."""
    return {k: c[k] for k in ("diag_kind", "alpha", "target") if k in c}


def options(c):
    if c["kind"] == "davidson":
        return dict(nroots=c["nroots"], max_p=c["max_p"], convergence_threshold=1e-8,
                    max_size_qspace=6 * c["nroots"], reset_D=8)
    o = dict(max_size_qspace=6, convergence_threshold=c["convergence_threshold"])
    if "max_iter" in c:
        o["max_iter"] = c["max_iter"]
    return o


# The CPU path re-run with its dots summed in other valid orders (oracle_ops.c or_set_sum_order):
# how far the REFERENCE algorithm itself moves under a change of rounding.
VARIANTS = {"reordered": 1,          # 8 interleaved partial sums (a vectorising build)
            "reordered_blocked": 2,  # 1024-element blocks folded pairwise (a blocked / threaded build)
            # the reference's distributed build on P MPI ranks with rank-order sums (rank-local sequential sums, partials
            # added in rank order: DistrArray.cpp:124-138 + MPI_Allreduce); generated for the RS cases
            # (--add-variants), whose residual norms move under them by more than under the two above
            "mpi2": 102, "mpi3": 103, "mpi4": 104, "mpi8": 108, "mpi16": 116}
DEFAULT_VARIANTS = ("reordered", "reordered_blocked")

# What each record pins, and the oracle revision that produced it (stamped into every record).
#   bit_exact  -- the GPU (short-vector arithmetic, exact_max raised where needed) and the CPU path must
#                 give these bits: C1 here, every record of mpi_traces.json / mpich_traces.json.  They
#                 change whenever the shared host algebra changes (iterative-solver_amd/include/itsolv_hbm/
#                 dense.h); all are regenerated here in seconds.
#   tolerance  -- N >= 2^21: held to the trace bar (tests/trace_check.py: same steps, eigenvalues to 1e-10,
#                 errors within the reference's own deviation under reordered sums), which absorbs valid
#                 re-roundings, including a revision of the host algebra; the N = 1e8 ones need a host with
#                 more memory than this container, so they keep the revision that produced them.
BIT_EXACT = ("C1_rank1", "C1_rank8")
# (A faster sym_eigen -- dlartg-form rotation radii, 4-sum tridiagonal dots: 20-30 % less host time --
# was tried in round 6 and not adopted: it moved the reference's own linear-equations criterion
# (test_LinearEquationsF.f90:80, residual <= 1e-4 on its ill-conditioned i+j+1 matrix, a value set by
# rounding) from 8.7e-5 to 1.04e-4 in one of the CPU path's summation-order variants.)
ORACLE_REVISION = "r5: dense.h sym_eigen with std::hypot rotation radii and sequential tridiagonal dots"


def stamp(name, rec, revision=ORACLE_REVISION):
    rec["parity"] = "bit_exact" if name in BIT_EXACT else "tolerance"
    rec["oracle_revision"] = revision
    return rec


def variant_record(c, r, v):
    """Deviation of variant run v from the reference run r (dict of trace arrays)."""
    import numpy as np

    tr, tv = r["trace"], v["trace"]
    k = min(len(tr["nq"]), len(tv["nq"]))
    return {
        "iterations": v["iterations"],
        "r_creations": v["r_creations"],
        "q_creations": v["q_creations"],
        "converged": v["converged"],
        "same_steps": bool(v["iterations"] == r["iterations"] and v["r_creations"] == r["r_creations"]
                           and list(tv["nq"]) == list(tr["nq"]) and list(tv["nwork"]) == list(tr["nwork"])
                           and list(tv.get("screened", [])) == list(tr.get("screened", []))),
        # per iteration (over the common prefix): max |error_variant - error_reference| over roots
        "error_abs_dev": np.max(np.abs(np.asarray(tv["errors"])[:k] - np.asarray(tr["errors"])[:k]),
                                axis=1).tolist(),
        "eigenvalue_rel_dev": (np.max(np.abs(np.asarray(tv["eigenvalues"])[:k] - np.asarray(tr["eigenvalues"])[:k])
                                      / np.maximum(np.abs(np.asarray(tr["eigenvalues"])[:k]), 1.0), axis=1).tolist()
                               if c["kind"] == "davidson" else []),
    }


def run(name, variants=DEFAULT_VARIANTS, base=None):
    """The reference run of case `name` (or `base`, its committed record) and the given variants."""
    import oracle

    c = CASES[name]
    t0 = time.time()
    fn = oracle.davidson_synthetic if c["kind"] == "davidson" else oracle.diis_synthetic
    runs = {}
    for key in variants:
        oracle.set_sum_order(VARIANTS[key])
        runs[key] = fn(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **problem_kw(c), **options(c))
    oracle.set_sum_order(0)
    if base is not None:
        out = dict(base)
        for key in variants:
            out[key] = variant_record(c, base, runs[key])
        return name, out
    r = fn(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **problem_kw(c), **options(c))
    tr = r["trace"]
    out = {
        "case": c,
        "options": options(c),
        "converged": r["converged"],
        "iterations": r["iterations"],
        "r_creations": r["r_creations"],
        "q_creations": r["q_creations"],
        "eigenvalues": [float(x) for x in r["eigenvalues"]] if c["kind"] == "davidson" else [],
        "errors": [float(x) for x in r["errors"]],
        "trace": {
            "eigenvalues": tr["eigenvalues"].tolist() if c["kind"] == "davidson" else [],
            "errors": tr["errors"].tolist(),
            "nq": tr["nq"].tolist(),
            "nwork": tr["nwork"].tolist(),
            "screened": tr["screened"].tolist(),
        },
        "redundant_params": r["redundant_params"],
        "null_params": r["null_params"],
        "cpu_seconds": round(time.time() - t0, 1),
    }
    for key in variants:
        out[key] = variant_record(c, r, runs[key])
    return name, stamp(name, out)


def _run_args(args):
    return run(*args)


PARTS = ("base",) + tuple(VARIANTS)


def run_part(name, part):
    """One run of case `name` in one process: the reference order ("base") or one variant; the raw
    trace (for hosts where the runs of a case do not fit in memory together: --part / --merge)."""
    import oracle

    c = CASES[name]
    t0 = time.time()
    fn = oracle.davidson_synthetic if c["kind"] == "davidson" else oracle.diis_synthetic
    oracle.set_sum_order(0 if part == "base" else VARIANTS[part])
    r = fn(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **problem_kw(c), **options(c))
    oracle.set_sum_order(0)
    tr = r["trace"]
    return {
        "case": name, "part": part, "converged": r["converged"], "iterations": r["iterations"],
        "r_creations": r["r_creations"], "q_creations": r["q_creations"],
        "eigenvalues": [float(x) for x in r["eigenvalues"]] if c["kind"] == "davidson" else [],
        "errors": [float(x) for x in r["errors"]],
        "trace": {"eigenvalues": tr["eigenvalues"].tolist() if c["kind"] == "davidson" else [],
                  "errors": tr["errors"].tolist(), "nq": tr["nq"].tolist(), "nwork": tr["nwork"].tolist(),
                  "screened": tr["screened"].tolist()},
        "redundant_params": r["redundant_params"], "null_params": r["null_params"],
        "cpu_seconds": round(time.time() - t0, 1),
    }


def merge_parts(parts):
    """The traces.json record of a case from its --part runs (one base, the variants)."""
    base = next(p for p in parts if p["part"] == "base")
    c = CASES[base["case"]]
    out = {"case": c, "options": options(c)}
    out.update({k: base[k] for k in ("converged", "iterations", "r_creations", "q_creations", "eigenvalues", "errors",
                                     "trace")})
    out["cpu_seconds"] = max(p["cpu_seconds"] for p in parts)
    for p in parts:
        if p["part"] != "base":
            out[p["part"]] = variant_record(c, base, p)
    return base["case"], stamp(base["case"], out)


# Short-vector cases for rank-order sums (tests/golden/mpi_traces.json): the whole solve record -- every
# trace value -- of the CPU path with its dots summed as P ranks' partials added in rank order (one
# valid MPI_Allreduce association), P = 1 (sequential), 2, 3, 4, 8.  On shards of at most
# ssp_ctx_set_exact_max elements the HIP path over a rank-order transport (peer memory, host hub) must
# reproduce them bit for bit (tests/dist_worker.py case gpu_exact_mpi).  MPICH's own association of the
# same cases: tests/golden/make_mpi_traces.py -> mpich_traces.json.
MPI_CASES = {
    "C1_rank1": CASES["C1_rank1"],
    "C1_rank8": CASES["C1_rank8"],
    "S_p8": {"kind": "davidson", "n": 10007, "rho": 0.1, "rank": 4, "seed": 20251015, "nroots": 4, "max_p": 8},
    "D_1000": {"kind": "diis", "n": 1000, "rho": 0.1, "rank": 1, "seed": 3},
}
MPI_ORDERS = {"mpi1": 0, "mpi2": 102, "mpi3": 103, "mpi4": 104, "mpi8": 108}


def mpi_options(c):
    if c["kind"] == "diis":
        return {"convergence_threshold": 1e-8, "max_size_qspace": 6}
    return {"nroots": c["nroots"], "max_p": c["max_p"], "convergence_threshold": 1e-8,
            "max_size_qspace": 6 * c["nroots"], "reset_D": 8}


def mpi_golden(out_path):
    import numpy as np

    import oracle

    out = {"_generator": "tests/golden/make_traces.py --mpi-golden: oracle (reference CPU path restated, "
                         "-ffp-contract=off), dots in the rank order of P MPI ranks",
           "_parity": "bit_exact", "_oracle_revision": ORACLE_REVISION}
    for name, c in MPI_CASES.items():
        fn = oracle.davidson_synthetic if c["kind"] == "davidson" else oracle.diis_synthetic
        rec = {"case": c, "options": mpi_options(c)}
        for key, order in MPI_ORDERS.items():
            oracle.set_sum_order(order)
            r = fn(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **mpi_options(c))
            tr = r["trace"]
            rec[key] = {"converged": r["converged"], "iterations": r["iterations"], "r_creations": r["r_creations"],
                        "q_creations": r["q_creations"], "eigenvalues": [float(x) for x in r["eigenvalues"]],
                        "errors": [float(x) for x in r["errors"]],
                        "residual_norms": [float(x) for x in r["residual_norms"]],
                        "trace": {k: np.asarray(tr[k]).tolist() for k in ("eigenvalues", "errors", "nq", "nwork",
                                                                          "screened")}}
            print(name, key, r["iterations"], r["r_creations"], flush=True)
        oracle.set_sum_order(0)
        out[name] = rec
    json.dump(out, open(out_path, "w"), indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mpi-golden", action="store_true", help="write tests/golden/mpi_traces.json")
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(HERE, "traces.json"))
    ap.add_argument("--omp", action="store_true",
                    help="the bit-identical OpenMP build of the CPU path (oracle/build/liboracle_itsolv_omp.so)")
    ap.add_argument("--add-variants", nargs="*", choices=list(VARIANTS),
                    help="only run these sum-order variants against the committed reference runs")
    ap.add_argument("--part", choices=PARTS, help="one run of the single --only case, written to --out as is")
    ap.add_argument("--merge", nargs="*", help="--part outputs of one case to merge into --out")
    a = ap.parse_args()
    if a.mpi_golden:
        mpi_golden(os.path.join(HERE, "mpi_traces.json"))
        return
    if a.omp:
        os.environ["ORACLE_OMP"] = "1"
    if a.part:
        (name,) = a.only
        r = run_part(name, a.part)
        json.dump(r, open(a.out, "w"))
        print(name, a.part, r["iterations"], r["r_creations"], r["cpu_seconds"], "s", flush=True)
        return
    if a.merge:
        name, rec = merge_parts([json.load(open(f)) for f in a.merge])
        old = json.load(open(a.out))
        old[name] = rec
        json.dump(dict(sorted(old.items())), open(a.out, "w"), indent=1)
        print(name, rec["iterations"], {k: rec[k]["same_steps"] for k in VARIANTS if k in rec}, flush=True)
        return
    names = a.only or [n for n in CASES if n != "C3_n1e8_rank8"]
    old = json.load(open(a.out)) if os.path.exists(a.out) else {}
    old = {k: v for k, v in old.items() if k in CASES or k.startswith("_")}
    variants = tuple(a.add_variants) if a.add_variants else DEFAULT_VARIANTS

    def job(n):
        return (n, variants, old[n]) if a.add_variants else (n, variants)

    # the N = 1e8 cases hold up to ~40 GB each: run them one at a time
    big = [n for n in names if CASES[n]["n"] >= 100_000_000]
    small = [n for n in names if n not in big]
    with ProcessPoolExecutor(a.jobs) as ex:
        for name, out in ex.map(_run_args, [job(n) for n in small]):
            old[name] = out
            print(name, out["iterations"], {k: out[k]["same_steps"] for k in VARIANTS if k in out}, flush=True)
    for n in big:
        name, out = run(*job(n))
        old[name] = out
        print(name, out["iterations"], {k: out[k]["same_steps"] for k in VARIANTS if k in out}, flush=True)
    old["_generator"] = ("tests/golden/make_traces.py: oracle (reference CPU path restated over "
                         "ArrayHandlerIterable loops, -ffp-contract=off)")
    json.dump(dict(sorted(old.items())), open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
