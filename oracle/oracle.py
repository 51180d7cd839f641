"""ORACLE — test infrastructure only.

ctypes binding of oracle/build/liboracle_ops.so (CPU restatement of the reference's
ArrayHandlerIterable kernels, see oracle_ops.h) plus numpy restatements of the synthetic problem.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker / the timed CPU baseline — never on the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle_ops.so")
_lib = None

PD = C.POINTER(C.c_double)
PZ = C.POINTER(C.c_size_t)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        Z, D, I, P = C.c_size_t, C.c_double, C.c_int, C.c_void_p
        sig = {
            "or_fill": [D, PD, Z],
            "or_scal": [D, PD, Z],
            "or_copy": [PD, Z, PD, Z],
            "or_axpy": [D, PD, Z, PD, Z],
            "or_dot": [PD, Z, PD, Z, PD],
            "or_gemm_inner": [P, I, P, I, Z, PD],
            "or_gemm_outer": [PD, P, I, P, I, Z],
            "or_select": [PD, Z, Z, I, I, PZ, PD, PZ],
            "or_select_max_dot": [PD, PD, Z, Z, PZ, PD, PZ],
            "or_sparse_copy": [PD, Z, PZ, PD, Z],
            "or_sparse_axpy": [D, PZ, PD, Z, PD, Z],
            "or_sparse_dot": [PD, Z, PZ, PD, Z, PD],
            "or_precondition": [P, I, PD, PD, Z],
            "or_distribution": [Z, I, PZ],
        }
        for name, args in sig.items():
            f = getattr(L, name)
            f.restype = C.c_int
            f.argtypes = args
        _lib = L
    return _lib


class OracleError(RuntimeError):
    pass


def _c(code):
    if code != 0:
        raise OracleError(f"oracle returned {code}")


def _d(a):
    return a.ctypes.data_as(PD)


def _z(a):
    return a.ctypes.data_as(PZ)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptrs(vs):
    return (C.c_void_p * max(1, len(vs)))(*[v.ctypes.data for v in vs])


def dot(x, y):
    x, y = _f64(x), _f64(y)
    out = C.c_double()
    _c(lib().or_dot(_d(x), x.size, _d(y), y.size, C.byref(out)))
    return out.value


def axpy(alpha, x, y):
    """Returns y + alpha * x (y is copied)."""
    x, y = _f64(x), _f64(y).copy()
    _c(lib().or_axpy(alpha, _d(x), x.size, _d(y), y.size))
    return y


def scal(alpha, x):
    x = _f64(x).copy()
    _c(lib().or_scal(alpha, _d(x), x.size))
    return x


def fill(alpha, n):
    x = np.empty(n)
    _c(lib().or_fill(alpha, _d(x), n))
    return x


def gemm_inner(xx, yy):
    xx = [_f64(v) for v in xx]
    yy = [_f64(v) for v in yy]
    out = np.zeros((len(xx), len(yy)))
    n = xx[0].size if xx else 0
    _c(lib().or_gemm_inner(_ptrs(xx), len(xx), _ptrs(yy), len(yy), n, _d(out)))
    return out


def gemm_outer(alphas, xx, yy):
    """Returns the updated copies of yy: yy[j] += sum_i alphas[i, j] xx[i] in reference order."""
    alphas = _f64(alphas)
    xx = [_f64(v) for v in xx]
    yy = [_f64(v).copy() for v in yy]
    n = yy[0].size if yy else 0
    _c(lib().or_gemm_outer(_d(alphas), _ptrs(xx), len(xx), _ptrs(yy), len(yy), n))
    return yy


def precondition(aa, d, shift):
    aa = [_f64(v).copy() for v in aa]
    d = _f64(d)
    sh = _f64(shift)
    _c(lib().or_precondition(_ptrs(aa), len(aa), _d(d), _d(sh), d.size))
    return aa


def select(x, nsel, max=False, ignore_sign=False):
    x = _f64(x)
    idx = np.zeros(max_(nsel), dtype=np.uint64)
    val = np.zeros(max_(nsel))
    nout = C.c_size_t()
    _c(lib().or_select(_d(x), x.size, nsel, int(max), int(ignore_sign), _z(idx), _d(val), C.byref(nout)))
    return idx[: nout.value].astype(np.int64), val[: nout.value]


def select_max_dot(x, y, nsel):
    x, y = _f64(x), _f64(y)
    idx = np.zeros(max_(nsel), dtype=np.uint64)
    val = np.zeros(max_(nsel))
    nout = C.c_size_t()
    _c(lib().or_select_max_dot(_d(x), _d(y), x.size, nsel, _z(idx), _d(val), C.byref(nout)))
    return idx[: nout.value].astype(np.int64), val[: nout.value]


def sparse_copy(n, idx, val):
    x = np.empty(n)
    idx = np.ascontiguousarray(idx, dtype=np.uint64)
    val = _f64(val)
    _c(lib().or_sparse_copy(_d(x), n, _z(idx), _d(val), idx.size))
    return x


def sparse_axpy(alpha, idx, val, y):
    y = _f64(y).copy()
    idx = np.ascontiguousarray(idx, dtype=np.uint64)
    val = _f64(val)
    _c(lib().or_sparse_axpy(alpha, _z(idx), _d(val), idx.size, _d(y), y.size))
    return y


def sparse_dot(x, idx, val):
    x = _f64(x)
    idx = np.ascontiguousarray(idx, dtype=np.uint64)
    val = _f64(val)
    out = C.c_double()
    _c(lib().or_sparse_dot(_d(x), x.size, _z(idx), _d(val), idx.size, C.byref(out)))
    return out.value


def distribution(dimension, nchunks):
    b = np.zeros(nchunks + 1, dtype=np.uint64)
    _c(lib().or_distribution(dimension, nchunks, _z(b)))
    return b.astype(np.int64)


def max_(n):
    return n if n > 0 else 1


# ORACLE_OMP=1: the bit-identical OpenMP build (elementwise loops and whole pairwise dots on several
# threads; make_traces.py --omp for the N = 1e8 traces)
ITSOLV_PATH = os.path.join(_HERE, "build", "liboracle_itsolv_omp.so" if os.environ.get("ORACLE_OMP") == "1"
                           else "liboracle_itsolv.so")
_itsolv = None


def itsolv_lib():
    """The reference CPU solver path (restated solvers + CPU handlers), oracle_* entry points."""
    global _itsolv
    if _itsolv is None:
        if not os.path.exists(ITSOLV_PATH):
            build()
        from itsolv_hbm import Options, Result, Synth  # struct layouts shared with the device library

        L = C.CDLL(ITSOLV_PATH)
        Z, D, I, U = C.c_size_t, C.c_double, C.c_int, C.c_ulonglong
        PO, PR, PDd = C.POINTER(Options), C.POINTER(Result), C.POINTER(C.c_double)
        for name, args in {
            "oracle_davidson_synthetic": [Z, D, I, U, PO, PR, PDd],
            "oracle_davidson_dense": [PDd, Z, PO, PR, PDd],
            "oracle_diis_synthetic": [Z, D, I, U, PO, PR, PDd],
            "oracle_diis_dense": [PDd, Z, PO, PR, PDd],
            "oracle_linear_equations_dense": [PDd, Z, PDd, I, PO, PR, PDd],
            "oracle_optimize_dense": [PDd, Z, I, PO, PR, PDd],
            "oracle_davidson_synth": [Z, C.POINTER(Synth), PO, PR, PDd],
            "oracle_diis_synth": [Z, C.POINTER(Synth), PO, PR, PDd],
        }.items():
            f = getattr(L, name)
            f.restype = I
            f.argtypes = args
        L.oracle_itsolv_last_error.restype = C.c_char_p
        P, LL = C.c_void_p, C.c_longlong
        L.oracle_rc_create.restype = P
        L.oracle_rc_create.argtypes = [C.c_char_p, Z, Z, PDd, D, D, I, C.c_char_p, C.c_char_p]
        L.oracle_rc_destroy.argtypes = [P]
        for name, args in {"oracle_rc_add_vector": [P, Z, PDd, PDd], "oracle_rc_add_value": [P, D, PDd, PDd],
                           "oracle_rc_end_iteration": [P, Z, PDd, PDd]}.items():
            getattr(L, name).restype = LL
            getattr(L, name).argtypes = args
        L.oracle_rc_add_p.restype = LL
        L.oracle_rc_add_p.argtypes = [P, Z, Z, C.POINTER(Z), C.POINTER(Z), PDd, PDd, PDd, PDd, C.c_void_p]
        L.oracle_rc_working_set_eigenvalues.restype = I
        L.oracle_rc_working_set_eigenvalues.argtypes = [P, PDd]
        for name in ("oracle_interpolate_cubic",):
            getattr(L, name).argtypes = [PDd, PDd, D, PDd]
        L.oracle_interpolate_minimize.argtypes = [PDd, PDd, D, D, PDd]
        L.oracle_interpolate_ex.restype = I
        L.oracle_interpolate_ex.argtypes = [PDd, PDd, C.c_char_p, D, D, D, Z, Z, I, PDd, PDd, PDd]
        L.oracle_test_problem_trig.restype = I
        L.oracle_test_problem_trig.argtypes = [Z, D, I]
        L.oracle_rc_solution.restype = I
        L.oracle_rc_solution.argtypes = [P, I, C.POINTER(C.c_int), PDd, PDd]
        L.oracle_rc_stats.restype = I
        L.oracle_rc_stats.argtypes = [P, C.POINTER(I), C.POINTER(I), PDd, PDd, PDd]
        _itsolv = L
    return _itsolv


def interpolate_cubic(p0, p1, x):
    """(x, f, f', f'') of the cubic through p0 = (x0, f0, g0), p1 (OptimizeBFGS's line-search model)."""
    out = np.zeros(4)
    itsolv_lib().oracle_interpolate_cubic(_d(np.array(p0, float)), _d(np.array(p1, float)), float(x), _d(out))
    return out


def interpolate_minimize(p0, p1, xa, xb):
    out = np.zeros(4)
    itsolv_lib().oracle_interpolate_minimize(_d(np.array(p0, float)), _d(np.array(p1, float)), float(xa), float(xb),
                                             _d(out))
    return out


def interpolate(p0, p1, interpolant="cubic", x=0.0, xa=0.0, xb=1.0, bracket_grid=100, max_bracket_grid=100000,
                analytic=True):
    """Interpolate(p0, p1, interpolant) (reference Interpolate.cpp:55-186): returns (the point at x,
    minimize(xa, xb, bracket_grid, max_bracket_grid, analytic), the four parameters), points as
    (x, f, f', f'')."""
    L = itsolv_lib()
    at, mn, par = np.zeros(4), np.zeros(4), np.zeros(4)
    if L.oracle_interpolate_ex(_d(np.array(p0, float)), _d(np.array(p1, float)), interpolant.encode(), float(x),
                               float(xa), float(xb), int(bracket_grid), int(max_bracket_grid), 1 if analytic else 0,
                               _d(at), _d(mn), _d(par)):
        raise RuntimeError(L.oracle_itsolv_last_error().decode())
    return at, mn, par


class RcSolver:
    """The reference CPU path behind the reverse-communication C API's call sequence
    (oracle_rc_*: the same solver construction and routing as iterative_solver_c.cpp, CPU
    handlers).  Method names and arguments follow iterative_solver.IterativeSolver."""

    def __init__(self, kind, n, nroot=1, rhs=None, thresh=1e-10, thresh_value=1e50, hermitian=True, algorithm="",
                 options=""):
        L = itsolv_lib()
        self.n, self.nroot = n, nroot
        b = None if rhs is None else np.ascontiguousarray(rhs, dtype=np.float64)
        self._h = L.oracle_rc_create(kind.encode(), n, nroot, None if b is None else _d(b), thresh, thresh_value,
                                     int(hermitian), algorithm.encode(), options.encode())
        if not self._h:
            raise RuntimeError(L.oracle_itsolv_last_error().decode())
        self._rhs = b

    def __del__(self):
        if getattr(self, "_h", None):
            itsolv_lib().oracle_rc_destroy(self._h)
            self._h = None

    def _r(self, v):
        if v < 0:
            raise RuntimeError(itsolv_lib().oracle_itsolv_last_error().decode())
        return int(v)

    @staticmethod
    def _nbuf(a):
        return a.shape[0] if a.ndim > 1 else 1

    def add_vector(self, parameters, action):
        return self._r(itsolv_lib().oracle_rc_add_vector(self._h, self._nbuf(parameters), _d(parameters), _d(action)))

    def add_value(self, value, parameters, action):
        return self._r(itsolv_lib().oracle_rc_add_value(self._h, float(value), _d(parameters), _d(action)))

    def end_iteration(self, parameters, residual):
        return self._r(itsolv_lib().oracle_rc_end_iteration(self._h, self._nbuf(parameters), _d(parameters),
                                                            _d(residual)))

    def add_p(self, pvectors, pp, parameters, action, apply_p):
        """As iterative_solver.IterativeSolver.add_p (IterativeSolverAddP)."""
        offsets = np.zeros(len(pvectors) + 1, dtype=np.uint64)
        idx, coef = [], []
        for k, p in enumerate(pvectors):
            for i in sorted(p):
                idx.append(i)
                coef.append(p[i])
            offsets[k + 1] = len(idx)
        idx = np.array(idx if idx else [0], dtype=np.uint64)
        coef = np.array(coef if coef else [0.0], dtype=np.float64)
        ppm = np.ascontiguousarray(pp, dtype=np.float64)
        n, nP = self.n, len(pvectors)
        fn_t = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_size_t, C.POINTER(C.c_size_t))

        def tramp(pbuf, gbuf, nvec, ranges):
            pc = np.ctypeslib.as_array(pbuf, shape=(nvec * nP,)).reshape(nvec, nP)
            rg = np.ctypeslib.as_array(ranges, shape=(2 * nvec,)).reshape(nvec, 2).astype(np.int64)
            g = np.ctypeslib.as_array(gbuf, shape=(nvec * n,))
            apply_p(pc, g, rg)

        self._apply_p = fn_t(tramp)
        Zp = C.POINTER(C.c_size_t)
        return self._r(itsolv_lib().oracle_rc_add_p(
            self._h, self._nbuf(parameters), nP, offsets.ctypes.data_as(Zp), idx.ctypes.data_as(Zp), _d(coef),
            _d(ppm), _d(parameters), _d(action), C.cast(self._apply_p, C.c_void_p)))

    def working_set_eigenvalues(self, nwork):
        ev = np.zeros(max(1, self.nroot))
        if itsolv_lib().oracle_rc_working_set_eigenvalues(self._h, _d(ev)):
            raise RuntimeError(itsolv_lib().oracle_itsolv_last_error().decode())
        return ev[:nwork]

    def solution(self, roots, parameters, residual):
        r = (C.c_int * max(1, len(roots)))(*roots)
        if itsolv_lib().oracle_rc_solution(self._h, len(roots), r, _d(parameters), _d(residual)):
            raise RuntimeError(itsolv_lib().oracle_itsolv_last_error().decode())

    def stats(self):
        it, rc = C.c_int(), C.c_int()
        err, ev, val = np.zeros(max(1, self.nroot)), np.zeros(max(1, self.nroot)), np.zeros(1)
        if itsolv_lib().oracle_rc_stats(self._h, C.byref(it), C.byref(rc), _d(err), _d(val), _d(ev)):
            raise RuntimeError(itsolv_lib().oracle_itsolv_last_error().decode())
        return {"iterations": it.value, "r_creations": rc.value, "errors": err[:self.nroot], "value": float(val[0]),
                "eigenvalues": ev[:self.nroot]}


def set_sum_order(order):
    """Summation order of the CPU path's dot / gemm_inner (oracle_ops.c or_set_sum_order): 0 = the
    reference's sequential loop (default), 1 = 8 interleaved partial sums (a vectorised build of the
    same loop), 2 = sequential sums over 1024-element blocks folded pairwise (a blocked / threaded
    reduction), 100 + P = the reference's distributed build on P MPI ranks (rank-local sequential
    sums, the P partials added in rank order).  Used only to measure the reference algorithm's own
    rounding sensitivity."""
    L = itsolv_lib()
    L.or_set_sum_order.argtypes = [C.c_int]
    L.or_set_sum_order.restype = C.c_int
    if L.or_set_sum_order(int(order)) != 0:
        raise ValueError(order)


def _solve(fn, args, nout):
    """nout == 0: no solution copy-back (null pointer)."""
    from itsolv_hbm import Result

    res = Result()
    out = np.zeros(max(1, nout))
    if fn(*args, C.byref(res), out.ctypes.data_as(PD) if nout > 0 else None) != 0:
        raise OracleError(itsolv_lib().oracle_itsolv_last_error().decode())
    return res.as_dict(), out


def davidson_synthetic(n, rho, rank, seed, solutions=True, *, diag_kind=0, alpha=0.0, target=1.0, **opts):
    from itsolv_hbm import Synth, make_options

    o = make_options(**opts)
    spec = Synth(rho, rank, seed, diag_kind, alpha, target)
    r, sol = _solve(itsolv_lib().oracle_davidson_synth, (n, C.byref(spec), C.byref(o)),
                    o.nroots * n if solutions else 0)
    if solutions:
        r["solutions"] = sol[: o.nroots * n].reshape(o.nroots, n)
    return r


def davidson_dense(h, **opts):
    from itsolv_hbm import make_options

    h = _f64(h)
    n = h.shape[0]
    o = make_options(**opts)
    r, sol = _solve(itsolv_lib().oracle_davidson_dense, (_d(h), n, C.byref(o)), o.nroots * n)
    r["solutions"] = sol[: o.nroots * n].reshape(o.nroots, n)
    return r


def diis_synthetic(n, rho, rank, seed, solutions=True, *, diag_kind=0, alpha=0.0, target=1.0, **opts):
    """diag_kind / alpha: the synthetic family (itsolv_hbm.DIAG_*, itsolv_hbm.c5_spec)."""
    from itsolv_hbm import Synth, make_options

    o = make_options(**opts)
    spec = Synth(rho, rank, seed, diag_kind, alpha, target)
    r, x = _solve(itsolv_lib().oracle_diis_synth, (n, C.byref(spec), C.byref(o)), n if solutions else 0)
    if solutions:
        r["x"] = x[:n]
    return r


def diis_dense(h, **opts):
    from itsolv_hbm import make_options

    h = _f64(h)
    n = h.shape[0]
    o = make_options(**opts)
    r, x = _solve(itsolv_lib().oracle_diis_dense, (_d(h), n, C.byref(o)), n)
    r["x"] = x[:n]
    return r


def linear_equations_dense(a, rhs, **opts):
    """The reference CPU path of LinearEquationsDavidson on A x_r = b_r (rows of rhs)."""
    from itsolv_hbm import make_options

    a = _f64(a)
    b = np.ascontiguousarray(np.atleast_2d(rhs), dtype=np.float64)
    n, nrhs = a.shape[0], b.shape[0]
    o = make_options(**opts)
    r, x = _solve(itsolv_lib().oracle_linear_equations_dense, (_d(a), n, _d(b), nrhs, C.byref(o)), n * nrhs)
    r["x"] = x[:n * nrhs].reshape(nrhs, n)
    return r


def optimize_dense(h, algorithm="BFGS", **opts):
    """The reference CPU path of OptimizeBFGS / OptimizeSD on the Rayleigh quotient of h from e_0."""
    from itsolv_hbm import make_options

    h = _f64(h)
    n = h.shape[0]
    o = make_options(**opts)
    r, x = _solve(itsolv_lib().oracle_optimize_dense, (_d(h), n, 0 if algorithm == "BFGS" else 1, C.byref(o)), n)
    r["x"] = x[:n]
    return r


class CpuUpdateStep:
    """bench.py's cpu_baseline leg: the reference CPU handler (ArrayHandlerIterable, pairwise
    gemm_inner/gemm_outer defaults) running bench.py's subspace-update op sequence in place."""

    def __init__(self, n, m, k, seed):
        self.n, self.m, self.k = n, m, k
        self.rp = [random_vector(n, seed, v) for v in range(m)]
        self.ra = [random_vector(n, seed, m + v) for v in range(m)]
        self.qp = [random_vector(n, seed, 2 * m + v) for v in range(k)]
        self.qa = [random_vector(n, seed, 2 * m + k + v) for v in range(k)]
        r = np.random.default_rng(seed)
        self.coef = np.ascontiguousarray(r.uniform(-0.1, 0.1, (k, m)))
        self.lam = r.uniform(0.5, 2.0, m)
        self.out = np.zeros((m, k))
        self.p_rp, self.p_ra, self.p_qp, self.p_qa = (_ptrs(v) for v in (self.rp, self.ra, self.qp, self.qa))

    def step(self):
        L, n, m, k = lib(), self.n, self.m, self.k
        _c(L.or_gemm_inner(self.p_rp, m, self.p_qp, k, n, _d(self.out)))
        _c(L.or_gemm_inner(self.p_rp, m, self.p_qa, k, n, _d(self.out)))
        for v in self.rp:
            _c(L.or_fill(0.0, _d(v), n))
        _c(L.or_gemm_outer(_d(self.coef), self.p_qp, k, self.p_rp, m, n))
        for v in self.ra:
            _c(L.or_fill(0.0, _d(v), n))
        _c(L.or_gemm_outer(_d(self.coef), self.p_qa, k, self.p_ra, m, n))
        for i in range(m):
            _c(L.or_axpy(-self.lam[i], _d(self.rp[i]), n, _d(self.ra[i]), n))
        out = C.c_double()
        for i in range(m):
            _c(L.or_dot(_d(self.ra[i]), n, _d(self.ra[i]), n, C.byref(out)))


def dram_resident_sample(seed=20251015):
    """One call each of the reference CPU loops on DRAM-resident operands (vectors far larger than
    the host caches): dot and axpy at N = 1e8, gemm_inner 8 x 48 (pairwise, gemm_inner_default) at
    N = 1e7.  Returns {op: {"n", "seconds", "bytes", "GBs"}} with the algorithmic bytes of SURVEY.md
    §8d (dot 16N, axpy 24N, gemm_inner 8N(m+k); the pairwise loop itself streams 2mk N 8 B)."""
    import time as _t

    L = lib()
    r = np.random.default_rng(seed)
    out = {}
    n = 100_000_000
    x, y = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    res = C.c_double()
    t0 = _t.perf_counter()
    _c(L.or_dot(_d(x), n, _d(y), n, C.byref(res)))
    dt = _t.perf_counter() - t0
    out["dot"] = {"n": n, "seconds": dt, "bytes": 16 * n, "GBs": 16 * n / dt / 1e9}
    t0 = _t.perf_counter()
    _c(L.or_axpy(0.5, _d(x), n, _d(y), n))
    dt = _t.perf_counter() - t0
    out["axpy"] = {"n": n, "seconds": dt, "bytes": 24 * n, "GBs": 24 * n / dt / 1e9}
    del x, y
    n, m, k = 10_000_000, 8, 48
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    ys = [r.uniform(-1, 1, n) for _ in range(k)]
    prod = np.zeros(m * k)
    t0 = _t.perf_counter()
    _c(L.or_gemm_inner(_ptrs(xs), m, _ptrs(ys), k, n, _d(prod)))
    dt = _t.perf_counter() - t0
    out["gemm_inner_8x48"] = {"n": n, "seconds": dt, "bytes": 8 * n * (m + k), "GBs": 8 * n * (m + k) / dt / 1e9,
                              "streamed_bytes": 16 * m * k * n}
    return out


class HostParallelStep:
    """bench.py's host-parallel baseline: the same op sequence with OpenMP over
    all host threads and cache-blocked gemm (oracle/host_parallel.c); not the reference's loops."""

    def __init__(self, n, m, k, seed):
        path = os.path.join(_HERE, "build", "libhost_parallel.so")
        if not os.path.exists(path):
            build()
        self.L = C.CDLL(path)
        self.L.hp_update_step.argtypes = [C.c_void_p] * 4 + [C.c_int, C.c_int, C.c_size_t] + [C.c_void_p] * 3
        self.L.hp_update_step.restype = C.c_int
        self.L.hp_first_touch.argtypes = [C.c_void_p, C.c_size_t, C.c_double]
        self.n, self.m, self.k = n, m, k
        self.vecs = []
        for v in range(2 * (m + k)):
            a = np.empty(n)
            self.L.hp_first_touch(a.ctypes.data, n, 1e-3 * (v + 1))
            self.vecs.append(a)
        self.p = [_ptrs(self.vecs[o:o + c]) for o, c in ((0, m), (m, m), (2 * m, k), (2 * m + k, k))]
        r = np.random.default_rng(seed)
        self.coef = np.ascontiguousarray(r.uniform(-0.1, 0.1, (k, m)))
        self.lam = r.uniform(0.5, 2.0, m)
        self.out = np.zeros(m * k)

    @property
    def threads(self):
        return int(self.L.hp_threads())

    def step(self):
        if self.L.hp_update_step(*[C.cast(p, C.c_void_p) for p in self.p], self.m, self.k, self.n,
                                 self.coef.ctypes.data, self.lam.ctypes.data, self.out.ctypes.data):
            raise RuntimeError("hp_update_step: shape beyond its limits")


# ---- synthetic problem restated in numpy (checker for sspx_*) ------------------------------------
_M64 = (1 << 64) - 1


def splitmix64(z):
    """Vectorised splitmix64 on uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def stream_key(seed, stream):
    with np.errstate(over="ignore"):
        s = np.uint64(seed) ^ (np.uint64(stream) * np.uint64(0xD1B54A32D192ED03))
    return splitmix64(s)


def random_vector(n, seed, vec, offset=0):
    g = np.arange(offset, offset + n, dtype=np.uint64)
    h = splitmix64(stream_key(seed, vec) ^ g)
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def synthetic_signs(n, rank, seed, offset=0):
    g = np.arange(offset, offset + n, dtype=np.uint64)
    u = np.ones((rank, n))
    for l in range(1, rank):
        h = splitmix64(stream_key(seed, 1000 + l) ^ g)
        u[l] = np.where((h & np.uint64(1)) != 0, -1.0, 1.0)
    return u


def synthetic_action(x, rho, rank, seed, offset=0):
    n = x.size
    u = synthetic_signs(n, rank, seed, offset)
    d = 1.0 + np.arange(offset, offset + n, dtype=np.float64)
    return d * x + rho * (u.T @ (u @ x))


def synthetic_diagonal(n, rho, rank, offset=0):
    return 1.0 + np.arange(offset, offset + n, dtype=np.float64) + rank * rho


def rank_one_eigenvalues(n, rho, nroots):
    """Exact lowest eigenvalues of diag(1..n) + rho*11^T (rho > 0) from the secular equation
    1 + rho * sum_i 1/(d_i - lam) = 0, one root in each (d_i, d_{i+1}), by bisection."""
    K = min(n, 4096)
    d = 1.0 + np.arange(K, dtype=np.float64)
    if n > K:
        from scipy.special import digamma  # sum_{i=K}^{n-1} 1/(i+1-lam) = psi(n+1-lam) - psi(K+1-lam)

        tail = lambda lam: digamma(n + 1.0 - lam) - digamma(K + 1.0 - lam)
    else:
        tail = lambda lam: 0.0
    roots = []
    for i in range(nroots):
        lo, hi = d[i], (d[i + 1] if i + 1 < n else d[i] + rho * n)
        f = lambda lam: 1.0 + rho * (np.sum(1.0 / (d - lam)) + tail(lam))
        a, b = lo + 1e-15 * max(1.0, abs(lo)), hi - 1e-15 * max(1.0, abs(hi))
        for _ in range(200):
            mid = 0.5 * (a + b)
            if f(mid) > 0:  # f increases from -inf to +inf across the interval
                b = mid
            else:
                a = mid
            if b - a <= 1e-15 * max(1.0, abs(mid)):
                break
        roots.append(0.5 * (a + b))
    return np.array(roots)
