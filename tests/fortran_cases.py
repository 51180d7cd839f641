"""Cases of the Fortran binding (module Iterative_Solver) for tests/test_fortran.py.

The Fortran callers live in tests/fortran/itsolv_f_checks.F90 (built by tests/fortran/Makefile):
libitsolv_f_checks.so calls the product library lib/libiterative_solver_f.so (the HIP path),
libitsolv_f_checks_emul.so the same module objects over oracle/build/libitsolv_emul.so (the C API
over the host emulation of the device ABI, no GPU).  `run_all(lib)` runs every case through one of
them and returns JSON-able results; `python tests/fortran_cases.py --emul OUT.json` writes the CPU
path's results for the GPU test to compare with (a separate process: the two libraries export the
same C API symbols): the reference arithmetic on the given inputs, and VARIANTS of it -- reordered
sums and fma-contracted multiply-adds (ssp_emul_set_arith: arithmetic a valid build of the
reference's loops may use) and inputs perturbed in their last bit (`perturb`) -- which tell the
cases whose steps the reference algorithm itself decides by rounding (a redundancy-screen argmax
between near-parallel residuals, a residual norm at the threshold).

Case lists follow the reference tests that call the Fortran test functions:
  eigen   test_LinearEigensystem.cpp:347-406 (file_eigen he/bh/hf with the 1e-8 degeneracy split,
          n_eigen n = 100, nonhermitian_eigen n = 6, small_eigen n = 1..4, symmetry_eigen n = 1..5;
          the Fortran test runs only np = 0, test_LinearEigensystemF.f90:21)
  lineq   test_LinearEquations.cpp:60-99 (symmetric_system n = 3..33, nroot < 14; rhs passed in the
          reference's memory layout, Problem_::rhs is an nroot x n column-major Eigen matrix)
  opt     test_Optimize.cpp:108-121 / test_OptimizeF.f90 (quadratic form, H = 1 + (i+2)*10 delta)
  diis    test_NonLinearEquations.cpp:111-117 (the same quadratic form with DIIS)
  solve   examples/LinearEigensystemExampleF-problem.F90, OptimizeExampleF-problem.F90
  pspace  examples/LinearEigensystemExampleF-Pspace.F90
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import rc_problems as rp  # noqa: E402

BUILD = os.path.join(HERE, "fortran", "build")
LIB_GPU = os.path.join(BUILD, "libitsolv_f_checks.so")
LIB_EMUL = os.path.join(BUILD, "libitsolv_f_checks_emul.so")

_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)
SZ = ctypes.c_size_t


def load(path):
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: run __graft_entry__.build() (needs /opt/rocm/bin/amdflang)")
    lib = ctypes.CDLL(path)
    lib.f_eigensystem.argtypes = [_D, SZ, SZ, ctypes.c_int, ctypes.c_double, ctypes.c_char_p, _D, _D, _I]
    lib.f_linear_equations.argtypes = [_D, _D, SZ, SZ, ctypes.c_double, ctypes.c_double, _D, _D]
    lib.f_optimize.argtypes = [_D, SZ, ctypes.c_int, ctypes.c_double, _D, _D]
    lib.f_diis.argtypes = [_D, SZ, ctypes.c_double, ctypes.c_char_p, _D, _D]
    lib.f_solve_matrix.argtypes = [_D, SZ, SZ, ctypes.c_double, ctypes.c_int, _D, _D]
    lib.f_solve_forced.argtypes = [SZ, ctypes.c_double, _D, _D]
    lib.f_pspace.argtypes = [_D, SZ, SZ, SZ, ctypes.c_double, _D, _D]
    for f in ("f_eigensystem", "f_linear_equations", "f_optimize", "f_diis", "f_solve_matrix", "f_solve_forced",
              "f_pspace", "f_mpi"):
        getattr(lib, f).restype = ctypes.c_int
    return lib


def _p(a):
    return a.ctypes.data_as(_D)


def perturb(a, seed):
    """a * (1 + 2^-52 r), r in {-1, 0, 1} per element (symmetric for a symmetric matrix); seed 0: a;
    seeds from 100: the uniform scaling a * (1 + (seed - 99) 2^-50)."""
    if seed == 0:
        return a
    if seed >= 100:
        return a * (1 + (seed - 99) * 2.0 ** -50)
    r = np.random.default_rng(seed).integers(-1, 2, a.shape).astype(float)
    if a.ndim == 2 and a.shape[0] == a.shape[1] and np.array_equal(a, a.T):
        r = np.triu(r) + np.triu(r, 1).T
    return a * (1 + 2.0 ** -52 * r)


def hamiltonian(name, split=1e-8):
    """load_matrix(file, degeneracy_split) (test_LinearEigensystem.cpp:53-63)."""
    with open(os.path.join(HERE, "golden", f"{name}.hamiltonian")) as f:
        t = f.read().split()
    n = int(t[0])
    h = np.array(t[1:1 + n * n], dtype=float).reshape(n, n)
    h[np.diag_indices(n)] += split * np.arange(n)
    return h


def eigen_matrices():
    out = [(f"file/{nm}", hamiltonian(nm)) for nm in ("he", "bh", "hf")]
    out.append(("n_eigen/100", rp.eigen_matrix(100, 1.0)))
    for param in (1.0, 0.1):
        for nh in (0.0, 0.1, 0.2):
            out.append((f"nonhermitian/6/{param}/{nh}", rp.eigen_matrix(6, param, nh)))
    for n in range(1, 5):
        out.append((f"small/{n}", rp.eigen_matrix(n, 1.0)))
    for n in range(1, 6):
        out.append((f"symmetry/{n}", rp.symmetry_matrix(n, 1.0)))
    return out


def lineq_problem(n, nroot):
    """Problem_ (test_LinearEquations.cpp:17-35): matrix i+j+1 (+1 on the diagonal), rhs row i =
    (i+1)(n(n+1)/2 + j n + 1), stored as the reference's nroot x n column-major Eigen matrix."""
    m = np.fromfunction(lambda i, j: i + j + 1.0, (n, n))
    m[np.diag_indices(n)] += 1.0
    rhs = np.array([[(i + 1) * (n * (n + 1) // 2 + j * n + 1) for j in range(n)] for i in range(nroot)], float)
    # the bytes of rhs.data() (column-major nroot x n), read by Fortran as rhs(n, nroot)
    rhs_f = np.asfortranarray(rhs).ravel(order="K").reshape((n, nroot), order="F")
    return m, np.asfortranarray(rhs_f)


def run_eigen(lib, h, nroot, hermitian, thresh=1e-8, options=""):
    n = h.shape[0]
    hf = np.asfortranarray(h)
    ev, err = np.zeros(nroot), np.zeros(nroot)
    rng = (ctypes.c_int * 2)()
    it = lib.f_eigensystem(_p(hf), n, nroot, int(hermitian), thresh, options.encode(), _p(ev), _p(err), rng)
    return {"iterations": it, "eigenvalues": ev.tolist(), "errors": err.tolist(), "range": [rng[0], rng[1]]}


def run_all(lib, seed=0):
    res = {}
    for name, h in eigen_matrices():
        n = h.shape[0]
        herm = bool(np.array_equal(h, h.T))
        for nroot, np_ in rp.eigen_cases(n, herm):
            if np_ == 0:
                res[f"eigen/{name}/{nroot}"] = run_eigen(lib, perturb(h, seed), nroot, herm)
    for n in range(3, 34, 3):
        for nroot in range(1, min(n, 13) + 1):
            m, rhs = lineq_problem(n, nroot)
            m, rhs = np.asfortranarray(perturb(m, seed)), np.asfortranarray(perturb(rhs, seed + 50 if 0 < seed < 100 else seed))
            sol, rn = np.zeros((n, nroot), order="F"), np.zeros(1)
            it = lib.f_linear_equations(_p(m), _p(rhs), n, nroot, 0.0, 1e-10, _p(sol), _p(rn))
            res[f"lineq/{n}/{nroot}"] = {"iterations": it, "solution": sol.ravel(order="F").tolist(),
                                         "residual": float(rn[0])}
    for n in (2, 11, 20, 29):
        h = np.asfortranarray(perturb(rp.quadratic_matrix(n, 10.0), seed))
        for code, alg in enumerate(("BFGS", "SD")):
            x, v = np.zeros(n), np.zeros(1)
            it = lib.f_optimize(_p(h), n, code, 1e-8, _p(x), _p(v))
            res[f"opt/{alg}/{n}"] = {"iterations": it, "x": x.tolist(), "value": float(v[0])}
    for n in (2, 7, 20, 50):
        h = np.asfortranarray(perturb(rp.quadratic_matrix(n, 10.0), seed))
        x, e = np.zeros(n), np.zeros(1)
        it = lib.f_diis(_p(h), n, 1e-8, b"max_size_qspace=6", _p(x), _p(e))
        res[f"diis/{n}"] = {"iterations": it, "x": x.tolist(), "error": float(e[0])}
    n, nroot = 1000, 5
    h = np.ones((n, n))
    h[np.diag_indices(n)] = 3.0 * np.arange(1, n + 1)
    hf = np.asfortranarray(perturb(h, seed))
    ev, err = np.zeros(nroot), np.zeros(nroot)
    it = lib.f_solve_matrix(_p(hf), n, nroot, 1e-7, 30, _p(ev), _p(err))
    res["solve/matrix"] = {"iterations": it, "eigenvalues": ev.tolist(), "errors": err.tolist()}
    x, v = np.zeros(5), np.zeros(1)
    quiet = lib.f_solve_forced(5, 1e-6, _p(x), _p(v))
    res["solve/forced"] = {"quiet": quiet, "x": x.tolist(), "value": float(v[0])}
    n, nroot, np_ = 200, 3, 30
    h = np.ones((n, n))
    h[np.diag_indices(n)] = 3.0 * np.arange(1, n + 1)
    hf = np.asfortranarray(perturb(h, seed))
    ev, err = np.zeros(nroot), np.zeros(nroot)
    it = lib.f_pspace(_p(hf), n, nroot, np_, 1e-8, _p(ev), _p(err))
    res["pspace"] = {"iterations": it, "eigenvalues": ev.tolist(), "errors": err.tolist()}
    res["mpi"] = {"size_rank": lib.f_mpi()}
    return res


# (sum order, fma, perturbation seed); the first is the reference arithmetic on the given inputs
VARIANTS = [(o, f, s) for s in (0, 1, 2, 100, 101) for o in (0, 1) for f in (0, 1)]


def set_arith(order, fma):
    """Arithmetic variant of the emulation's reductions and multiply-adds (ssp_emul_set_arith)."""
    emul = ctypes.CDLL(os.path.join(HERE, "..", "oracle", "build", "libssp_emul.so"))
    if emul.ssp_emul_set_arith(ctypes.c_int(order), ctypes.c_int(fma)) != 0:
        raise ValueError((order, fma))


if __name__ == "__main__":
    if len(sys.argv) != 3 or sys.argv[1] != "--emul":
        sys.exit("usage: fortran_cases.py --emul OUT.json")
    lib = load(LIB_EMUL)
    out = {}
    for order, fma, seed in VARIANTS:
        set_arith(order, fma)
        out[f"{order}/{fma}/{seed}"] = run_all(lib, seed)
    with open(sys.argv[2], "w") as f:
        json.dump(out, f)
