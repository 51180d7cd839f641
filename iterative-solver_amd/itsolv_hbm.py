"""ctypes binding of libitsolv_hbm.so (C ABI: include/itsolv_hbm.h): the restated Davidson / DIIS
solvers running over the HBM handlers.  The options / result structures are shared with the
oracle's CPU twin (oracle/itsolv_oracle.cpp)."""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

import subspace_hip as sh

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libitsolv_hbm.so")
MAX_ROOTS = 64
TRACE_ITER, TRACE_ROOTS = 256, 8

EXPORTS = [
    "itsolv_last_error", "itsolv_default_options", "itsolv_davidson_synthetic", "itsolv_davidson_dense",
    "itsolv_diis_synthetic", "itsolv_diis_dense", "itsolv_linear_equations_dense", "itsolv_optimize_dense",
    "itsolv_davidson_synth", "itsolv_diis_synth",
]

# Diagonal families of the synthetic H (include/subspace_hip.h sspx_synth, itsolv_hbm/problems.h).
DIAG_LINEAR, DIAG_BOUNDED = 0, 1


class Synth(C.Structure):
    _fields_ = [("rho", C.c_double), ("rank", C.c_int), ("seed", C.c_ulonglong), ("diag_kind", C.c_int),
                ("alpha", C.c_double), ("target", C.c_double)]


def c5_spec(n: int, rank: int = 1, seed: int = 3, alpha: float = 0.2) -> dict:
    """BASELINE config C5's well-posed DIIS instance (itsolv_hbm/problems.h c5_spec): r = H (x - t 1),
    H = diag(1 + 2 frac(g phi1)) + (1/n) sum_l u_l u_l^T, preconditioner diagonal mismatched by alpha,
    t = 1/sqrt(n) (a unit-norm solution).  Keyword arguments of diis_synthetic / oracle.diis_synthetic."""
    return dict(rho=1.0 / n, rank=rank, seed=seed, diag_kind=DIAG_BOUNDED, alpha=alpha, target=1.0 / math.sqrt(n))


class Options(C.Structure):
    _fields_ = [
        ("nroots", C.c_int),
        ("nwork", C.c_int),
        ("max_iter", C.c_int),
        ("max_size_qspace", C.c_int),
        ("reset_D", C.c_int),
        ("reset_D_max_Q_size", C.c_int),
        ("max_p", C.c_int),
        ("p_threshold", C.c_double),
        ("convergence_threshold", C.c_double),
        ("hermitian", C.c_int),
        ("generate_initial_guess", C.c_int),
        ("verbosity", C.c_int),
        ("augmented_hessian", C.c_double),
        ("block_gram_schmidt", C.c_int),
    ]


class Result(C.Structure):
    _fields_ = [
        ("converged", C.c_int),
        ("iterations", C.c_int),
        ("r_creations", C.c_int),
        ("q_creations", C.c_int),
        ("nroots", C.c_int),
        ("eigenvalues", C.c_double * MAX_ROOTS),
        ("errors", C.c_double * MAX_ROOTS),
        ("residual_norms", C.c_double * MAX_ROOTS),
        ("seconds", C.c_double),
        ("n_eig_trace", C.c_int),
        ("eig_trace", C.c_double * 256),
        ("trace_roots", C.c_int),
        ("trace_nq", C.c_int * TRACE_ITER),
        ("trace_nwork", C.c_int * TRACE_ITER),
        ("trace_eigenvalues", C.c_double * (TRACE_ITER * TRACE_ROOTS)),
        ("trace_errors", C.c_double * (TRACE_ITER * TRACE_ROOTS)),
        ("redundant_params", C.c_int),
        ("null_params", C.c_int),
        ("trace_screened", C.c_int * TRACE_ITER),
        ("host_algebra_seconds", C.c_double),
        ("host_algebra_calls", C.c_int),
        ("host_algebra_max_dim", C.c_int),
    ]

    def as_dict(self):
        k = self.nroots
        return {
            "converged": bool(self.converged),
            "iterations": self.iterations,
            "r_creations": self.r_creations,
            "q_creations": self.q_creations,
            "redundant_params": self.redundant_params,
            "null_params": self.null_params,
            "eigenvalues": np.array(self.eigenvalues[:k]),
            "errors": np.array(self.errors[:k]),
            "residual_norms": np.array(self.residual_norms[:k]),
            "seconds": self.seconds,
            "host_algebra": {"seconds": self.host_algebra_seconds, "calls": self.host_algebra_calls,
                             "max_dim": self.host_algebra_max_dim},
            "eig_trace": np.array(self.eig_trace[: self.n_eig_trace]),
            "trace": self.trace(),
        }

    def trace(self):
        """Per-iteration parity observables: one entry per solve() iteration."""
        it, nr = self.n_eig_trace, self.trace_roots
        ev = np.array(self.trace_eigenvalues[: it * TRACE_ROOTS]).reshape(it, TRACE_ROOTS)[:, :nr]
        er = np.array(self.trace_errors[: it * TRACE_ROOTS]).reshape(it, TRACE_ROOTS)[:, :nr]
        return {"eigenvalues": ev, "errors": er, "nq": np.array(self.trace_nq[:it]),
                "nwork": np.array(self.trace_nwork[:it]), "screened": np.array(self.trace_screened[:it])}


def make_options(**kw) -> Options:
    o = Options(nroots=1, nwork=0, max_iter=100, max_size_qspace=0, reset_D=0, reset_D_max_Q_size=0, max_p=0,
                p_threshold=0.0, convergence_threshold=1e-8, hermitian=1, generate_initial_guess=1, verbosity=0,
                augmented_hessian=0.0, block_gram_schmidt=-1)
    for k, v in kw.items():
        if not hasattr(o, k):
            raise KeyError(k)
        setattr(o, k, v)
    return o


_lib = None


def load_library():
    global _lib
    if _lib is None:
        sh.load_library()  # libsubspace_hip.so first (dependency, RTLD_GLOBAL)
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C iterative-solver_amd`")
        L = C.CDLL(LIB_PATH)
        P, Z, D, I, U = C.c_void_p, C.c_size_t, C.c_double, C.c_int, C.c_ulonglong
        PO, PR, PD = C.POINTER(Options), C.POINTER(Result), C.POINTER(C.c_double)
        sig = {
            "itsolv_last_error": (C.c_char_p, []),
            "itsolv_default_options": (None, [PO]),
            "itsolv_davidson_synthetic": (I, [P, Z, D, I, U, PO, PR, PD]),
            "itsolv_davidson_dense": (I, [P, PD, Z, PO, PR, PD]),
            "itsolv_diis_synthetic": (I, [P, Z, D, I, U, PO, PR, PD]),
            "itsolv_diis_dense": (I, [P, PD, Z, PO, PR, PD]),
            "itsolv_linear_equations_dense": (I, [P, PD, Z, PD, I, PO, PR, PD]),
            "itsolv_optimize_dense": (I, [P, PD, Z, I, PO, PR, PD]),
            "itsolv_davidson_synth": (I, [P, Z, C.POINTER(Synth), PO, PR, PD]),
            "itsolv_diis_synth": (I, [P, Z, C.POINTER(Synth), PO, PR, PD]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _call(fn, args, nout):
    res = Result()
    out = np.zeros(max(1, nout))
    # nout == 0: no solution copy-back (null pointer; the C side then skips the download)
    ptr = out.ctypes.data_as(C.POINTER(C.c_double)) if nout > 0 else None
    code = fn(*args, C.byref(res), ptr)
    if code != 0:
        raise RuntimeError(f"{fn.__name__}: {load_library().itsolv_last_error().decode()}")
    return res.as_dict(), out


def davidson_synthetic(ctx: sh.Context, n: int, rho: float, rank: int, seed: int, n_local: int | None = None,
                       solutions: bool = True, *, diag_kind: int = DIAG_LINEAR, alpha: float = 0.0,
                       target: float = 1.0, **opts):
    o = make_options(**opts)
    nl = n if n_local is None else n_local
    spec = Synth(rho, rank, seed, diag_kind, alpha, target)
    r, sol = _call(load_library().itsolv_davidson_synth, (ctx.handle, n, C.byref(spec), C.byref(o)),
                   o.nroots * nl if solutions else 0)
    if solutions:
        r["solutions"] = sol[: o.nroots * nl].reshape(o.nroots, nl)
    return r


def davidson_dense(ctx: sh.Context, h: np.ndarray, **opts):
    h = np.ascontiguousarray(h, dtype=np.float64)
    n = h.shape[0]
    o = make_options(**opts)
    r, sol = _call(load_library().itsolv_davidson_dense,
                   (ctx.handle, h.ctypes.data_as(C.POINTER(C.c_double)), n, C.byref(o)), o.nroots * n)
    r["solutions"] = sol[: o.nroots * n].reshape(o.nroots, n)
    return r


def diis_synthetic(ctx: sh.Context, n: int, rho: float, rank: int, seed: int, n_local: int | None = None,
                   solutions: bool = True, *, diag_kind: int = DIAG_LINEAR, alpha: float = 0.0,
                       target: float = 1.0, **opts):
    o = make_options(**opts)
    nl = n if n_local is None else n_local
    spec = Synth(rho, rank, seed, diag_kind, alpha, target)
    r, x = _call(load_library().itsolv_diis_synth, (ctx.handle, n, C.byref(spec), C.byref(o)),
                 nl if solutions else 0)
    if solutions:
        r["x"] = x[:nl]
    return r


def diis_dense(ctx: sh.Context, h: np.ndarray, **opts):
    h = np.ascontiguousarray(h, dtype=np.float64)
    n = h.shape[0]
    o = make_options(**opts)
    r, x = _call(load_library().itsolv_diis_dense, (ctx.handle, h.ctypes.data_as(C.POINTER(C.c_double)), n,
                                                    C.byref(o)), n)
    r["x"] = x[:n]
    return r


def linear_equations_dense(ctx: sh.Context, a: np.ndarray, rhs: np.ndarray, **opts):
    """LinearEquationsDavidson on A x_r = b_r (rows of rhs); returns the result dict with "x"."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(np.atleast_2d(rhs), dtype=np.float64)
    n, nrhs = a.shape[0], b.shape[0]
    o = make_options(**opts)
    r, x = _call(load_library().itsolv_linear_equations_dense,
                 (ctx.handle, a.ctypes.data_as(C.POINTER(C.c_double)), n, b.ctypes.data_as(C.POINTER(C.c_double)),
                  nrhs, C.byref(o)), n * nrhs)
    r["x"] = x[:n * nrhs].reshape(nrhs, n)
    return r


def optimize_dense(ctx: sh.Context, h: np.ndarray, algorithm: str = "BFGS", **opts):
    """OptimizeBFGS / OptimizeSD on the Rayleigh quotient of h from e_0 (function value in eigenvalues[0])."""
    h = np.ascontiguousarray(h, dtype=np.float64)
    n = h.shape[0]
    o = make_options(**opts)
    r, x = _call(load_library().itsolv_optimize_dense,
                 (ctx.handle, h.ctypes.data_as(C.POINTER(C.c_double)), n, 0 if algorithm == "BFGS" else 1,
                  C.byref(o)), n)
    r["x"] = x[:n]
    return r
