"""iterative_solver on MI355X: the reference's Python API (python/iterative_solver, a Cython
extension over src/molpro/linalg/IterativeSolverC.h) as a ctypes binding of the same C API in
libitsolv_hbm.so (include/iterative_solver_c.h).  Class names, constructor arguments and methods
follow the reference (iterative_solver_extension.pyx); the Q space and all subspace operations
live in HBM, the parameter/residual arrays the caller passes stay numpy arrays.

Available: LinearEigensystem and LinearEquations (Davidson), NonLinearEquations (DIIS), Optimize
(BFGS, SD).
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

from .problem import Problem

__all__ = ["Problem", "IterativeSolver", "LinearEigensystem", "NonLinearEquations", "LinearEquations", "Optimize"]

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_HERE, "lib", "libitsolv_hbm.so")
_lib = None

P, D, Z, I = C.c_void_p, C.c_double, C.c_size_t, C.c_int
PD, PZ, PI = C.POINTER(C.c_double), C.POINTER(C.c_size_t), C.POINTER(C.c_int)
APPLY_P = C.CFUNCTYPE(None, PD, PD, C.c_size_t, PZ)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C iterative-solver_amd`")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        sig = {
            "IterativeSolverLinearEigensystemInitialize": (None, [Z, Z, PZ, PZ, D, D, I, I, C.c_char_p, C.c_int64,
                                                                  C.c_char_p, C.c_char_p]),
            "IterativeSolverLinearEquationsInitialize": (None, [Z, Z, PZ, PZ, PD, D, D, D, I, I, C.c_char_p, C.c_int64,
                                                                C.c_char_p, C.c_char_p]),
            "IterativeSolverNonLinearEquationsInitialize": (None, [Z, PZ, PZ, D, I, C.c_char_p, C.c_int64, C.c_char_p,
                                                                   C.c_char_p]),
            "IterativeSolverOptimizeInitialize": (None, [Z, PZ, PZ, D, D, I, I, C.c_char_p, C.c_int64, C.c_char_p,
                                                         C.c_char_p]),
            "IterativeSolverFinalize": (None, []),
            "IterativeSolverAddVector": (Z, [Z, PD, PD, I]),
            "IterativeSolverSolution": (None, [I, PI, PD, PD, I]),
            "IterativeSolverAddValue": (Z, [D, PD, PD, I]),
            "IterativeSolverEndIteration": (Z, [Z, PD, PD, I]),
            "IterativeSolverEndIterationNeeded": (I, []),
            "IterativeSolverAddP": (Z, [Z, Z, PZ, PZ, PD, PD, PD, PD, I, APPLY_P]),
            "IterativeSolverErrors": (None, [PD]),
            "IterativeSolverEigenvalues": (None, [PD]),
            "IterativeSolverWorkingSetEigenvalues": (None, [PD]),
            "IterativeSolverSuggestP": (Z, [PD, PD, Z, D, PZ]),
            "IterativeSolverPrintStatistics": (None, []),
            "IterativeSolverNonLinear": (I, []),
            "IterativeSolverHasValues": (I, []),
            "IterativeSolverHasEigenvalues": (I, []),
            "IterativeSolverSetDiagonals": (None, [PD]),
            "IterativeSolverDiagonals": (None, [PD]),
            "IterativeSolverValue": (D, []),
            "IterativeSolverVerbosity": (I, []),
            "IterativeSolverMaxIter": (I, []),
            "IterativeSolverSetMaxIter": (None, [I]),
            "IterativeSolver_mpicomm_global": (C.c_int64, []),
            "IterativeSolverHbmSetContext": (I, [P]),
            "IterativeSolverHbmSetThrow": (I, [I]),
            "IterativeSolverHbmStatistics": (I, [PI, PI, PI]),
            "IterativeSolverHbmLastError": (C.c_char_p, []),
            "IterativeSolverHbmInstanceId": (C.c_uint64, []),
            "IterativeSolverHbmFinalizeInstance": (I, [C.c_uint64]),
            "IterativeSolverHbmMpiActive": (I, []),
            "IterativeSolverHbmMpiAttach": (I, [P, C.c_int64, C.c_char_p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        lib.IterativeSolverHbmSetThrow(0)  # ctypes cannot unwind C++ exceptions: record them instead
        _lib = lib
    return _lib


def _call(name, *args):
    lib = _load()
    r = getattr(lib, name)(*args)
    err = lib.IterativeSolverHbmLastError()
    if err:
        raise RuntimeError(err.decode())
    return r


def _d(a):
    return a.ctypes.data_as(PD)


def use_context(ctx):
    """Run the instances created after this call on `ctx` (a subspace_hip.Context, possibly with a
    communicator attached); None restores the default single-rank context on device 0."""
    _call("IterativeSolverHbmSetContext", ctx.handle if ctx is not None else None)


def statistics():
    it, r, q = C.c_int(), C.c_int(), C.c_int()
    if _load().IterativeSolverHbmStatistics(C.byref(it), C.byref(r), C.byref(q)) != 0:
        raise RuntimeError("no active solver")
    return {"iterations": it.value, "r_creations": r.value, "q_creations": q.value}


def _flat(a):
    if not (a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]):
        raise ValueError("parameter/residual arrays must be C-contiguous float64")
    return a


class IterativeSolver:
    """Base of LinearEigensystem / NonLinearEquations (reference iterative_solver_extension.pyx)."""

    def __init__(self, n, nroot=1):
        self.n = n
        self.nroot = nroot
        self.value = None
        self._id = 0

    def _register(self):
        """Called after the C layer pushed this object's instance: remember its id."""
        self._id = int(_load().IterativeSolverHbmInstanceId())
        self._active = self._id != 0

    def _check_top(self):
        # The C layer drives its top instance only (reference IterativeSolverCMPI.cpp); a call
        # through an older object while a newer one is alive would silently drive the newer one.
        if not getattr(self, "_active", False):
            raise RuntimeError("this solver has been finalized")
        if int(_load().IterativeSolverHbmInstanceId()) != self._id:
            raise RuntimeError("another IterativeSolver instance is active (created later and not finalized)")

    def __del__(self):
        # Removes this object's own instance wherever it is in the C layer's stack, never another's.
        try:
            if getattr(self, "_active", False):
                _load().IterativeSolverHbmFinalizeInstance(self._id)
                self._active = False
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def mpicomm_compute(self):
        """The communicator the instances use by default, as in the reference
        (iterative_solver_extension.pyx:27-31): IterativeSolver_mpicomm_global(), the Fortran handle of
        MPI_COMM_WORLD when the process has initialised MPI (the C layer then shards the vectors over its
        ranks), else 0 (no communicator: one rank, or the context set by use_context)."""
        return _mpicomm_compute()

    def finalize(self):
        if getattr(self, "_active", False):
            _load().IterativeSolverHbmFinalizeInstance(self._id)
            self._active = False

    def solution(self, roots, parameters, residual, sync=True):
        self._check_top()
        roots_ = (C.c_int * max(1, len(roots)))(*roots)
        _call("IterativeSolverSolution", len(roots), roots_, _d(_flat(parameters)), _d(_flat(residual)), int(sync))
        return self.value

    def add_vector(self, parameters, action, sync=True):
        self._check_top()
        nbuffer = parameters.shape[0] if parameters.ndim > 1 else 1
        return int(_call("IterativeSolverAddVector", nbuffer, _d(_flat(parameters)), _d(_flat(action)), int(sync)))

    def add_value(self, value, parameters, action, sync=True):
        self._check_top()
        r = int(_call("IterativeSolverAddValue", value, _d(_flat(parameters)), _d(_flat(action)), int(sync)))
        self.value = value
        return r

    def end_iteration(self, parameters, residual, sync=True):
        self._check_top()
        nbuffer = parameters.shape[0] if parameters.ndim > 1 else 1
        return int(_call("IterativeSolverEndIteration", nbuffer, _d(_flat(parameters)), _d(_flat(residual)),
                         int(sync)))

    def add_p(self, pvectors, pp, parameters, action, apply_p, sync=True):
        """P space from sparse vectors [{index: coefficient}], the P-P action matrix `pp` (nP x nP)
        and a callback apply_p(p_coefficients (nvec x nP), actions_local, ranges) that adds the P
        contributions to this rank's range of the action rows (reference IterativeSolverAddP)."""
        self._check_top()
        offsets = np.zeros(len(pvectors) + 1, dtype=np.uint64)
        idx, coef = [], []
        for k, p in enumerate(pvectors):
            for i in sorted(p):
                idx.append(i)
                coef.append(p[i])
            offsets[k + 1] = len(idx)
        idx = np.array(idx, dtype=np.uint64)
        coef = np.array(coef, dtype=np.float64)
        ppm = np.ascontiguousarray(pp, dtype=np.float64)
        n, nP = self.n, len(pvectors)

        def tramp(pbuf, gbuf, nvec, ranges):
            pc = np.ctypeslib.as_array(pbuf, shape=(nvec * nP,)).reshape(nvec, nP)
            rg = np.ctypeslib.as_array(ranges, shape=(2 * nvec,)).reshape(nvec, 2).astype(np.int64)
            # gbuf points at element range[0] of action row 0; rows are n apart.
            g = np.ctypeslib.as_array(gbuf, shape=((nvec - 1) * n + (rg[-1, 1] - rg[-1, 0]),))
            apply_p(pc, g, rg)

        self._apply_p = APPLY_P(tramp)  # keep alive for the solver's lifetime
        nbuffer = parameters.shape[0] if parameters.ndim > 1 else 1
        return int(_call("IterativeSolverAddP", nbuffer, nP, offsets.ctypes.data_as(PZ), idx.ctypes.data_as(PZ),
                         _d(coef), _d(ppm), _d(_flat(parameters)), _d(_flat(action)), int(sync), self._apply_p))

    @property
    def end_iteration_needed(self):
        self._check_top()
        return _call("IterativeSolverEndIterationNeeded") != 0

    @property
    def errors(self):
        self._check_top()
        e = np.zeros(self.nroot)
        _call("IterativeSolverErrors", _d(e))
        return e

    def working_set_eigenvalues(self, nwork):
        self._check_top()
        ev = np.zeros(max(1, self.nroot))
        _call("IterativeSolverWorkingSetEigenvalues", _d(ev))
        return ev[:nwork]

    def statistics(self):
        self._check_top()
        return statistics()

    def solve(self, parameters, actions, problem, generate_initial_guess=False, max_iter=None):
        """One-call driver over the reverse-communication API, the loop of the reference's
        IterativeSolver.solve (iterative_solver_extension.pyx:78-165)."""
        self._check_top()
        if parameters.ndim < 2 or actions.ndim < 2:
            return self.solve(parameters.reshape([self.nroot, self.n]), actions.reshape([self.nroot, self.n]), problem,
                              generate_initial_guess, max_iter)
        nbuffer = parameters.shape[0]
        ev = np.zeros(self.nroot)
        errors = np.zeros(self.nroot)
        verbosity = _call("IterativeSolverVerbosity")
        use_diagonals = problem.diagonals(actions.reshape([actions.size]))
        if max_iter is not None:
            _call("IterativeSolverSetMaxIter", int(max_iter))
        if use_diagonals:
            _call("IterativeSolverSetDiagonals", _d(actions))
        if generate_initial_guess:
            parameters[:, :] = 0
            if isinstance(self, LinearEigensystem):
                if not use_diagonals:
                    raise ValueError("Default initial guess requested, but diagonal elements are not available")
                _call("IterativeSolverDiagonals", _d(actions))
                for i in range(self.nroot):
                    argmin = int(np.argmin(actions[0, :]))
                    actions[0, argmin] = sys.float_info.max
                    parameters[i, argmin] = 1.0
            elif isinstance(self, LinearEquations):
                for i in range(self.nroot):
                    parameters[i, i] = 1
        nwork = nbuffer
        value = None
        for it in range(_call("IterativeSolverMaxIter")):
            if _call("IterativeSolverNonLinear") > 0:
                value = problem.residual(parameters.reshape([parameters.shape[-1]]),
                                         actions.reshape([parameters.shape[-1]]))
                if isinstance(self, Optimize):
                    nwork = self.add_value(value, parameters, actions)
                else:
                    nwork = self.add_vector(parameters[0, :], actions[0, :])
            else:
                problem.action(parameters, actions)
                nwork = self.add_vector(parameters[:nwork, :], actions[:nwork, :])
            while self.end_iteration_needed:
                if nwork > 0:
                    _call("IterativeSolverWorkingSetEigenvalues", _d(ev))
                    if use_diagonals:
                        _call("IterativeSolverDiagonals", _d(parameters))
                        problem.precondition(actions[:nwork, :], shift=ev[:nwork],
                                             diagonals=parameters.reshape([parameters.size])[:parameters.shape[-1]])
                    else:
                        problem.precondition(actions[:nwork, :], shift=ev[:nwork])
                nwork = self.end_iteration(parameters, actions)
            _call("IterativeSolverErrors", _d(errors))
            self.value = _call("IterativeSolverValue")
            if _call("IterativeSolverHasValues") != 0:
                reported = problem.report(it + 1 if nwork > 0 else 0, verbosity, errors, value=value)
            elif _call("IterativeSolverHasEigenvalues") != 0:
                _call("IterativeSolverEigenvalues", _d(ev))
                reported = problem.report(it + 1 if nwork > 0 else 0, verbosity, errors, eigenvalues=ev[:self.nroot])
            else:
                reported = problem.report(it + 1 if nwork > 0 else 0, verbosity, errors)
            if not reported and verbosity >= 2:
                print("Iteration", it, "log10(|residual|)=", np.log10(errors))
            if nwork < 1:
                break


_m_mpicomm_compute = None


def _mpicomm_compute():
    global _m_mpicomm_compute
    if _m_mpicomm_compute is None:
        _m_mpicomm_compute = int(_call("IterativeSolver_mpicomm_global"))
    return _m_mpicomm_compute


def _comm(mpicomm):
    return int(mpicomm) if mpicomm is not None else _mpicomm_compute()


def _range_arrays(range):
    rb = C.c_size_t(range[0] if range is not None else 0)
    re = C.c_size_t(range[1] if range is not None else 0)
    return rb, re


class LinearEigensystem(IterativeSolver):
    def __init__(self, n, nroot, range=None, thresh=1e-10, thresh_value=1e50, hermitian=False, verbosity=0,
                 pname="", mpicomm=None, algorithm="", options=""):
        super().__init__(n, nroot)
        rb, re = _range_arrays(range)
        _call("IterativeSolverLinearEigensystemInitialize", n, nroot, C.byref(rb), C.byref(re), thresh, thresh_value,
              1 if hermitian else 0, verbosity, pname.encode(), _comm(mpicomm), algorithm.encode(),
              options.encode())
        self._register()
        if range is not None:
            range[0], range[1] = rb.value, re.value

    @property
    def eigenvalues(self):
        self._check_top()
        e = np.zeros(self.nroot)
        _call("IterativeSolverEigenvalues", _d(e))
        return e


class NonLinearEquations(IterativeSolver):
    def __init__(self, n, range=None, thresh=1e-10, verbosity=0, pname="", mpicomm=None, algorithm="", options=""):
        super().__init__(n)
        rb, re = _range_arrays(range)
        _call("IterativeSolverNonLinearEquationsInitialize", n, C.byref(rb), C.byref(re), thresh, verbosity,
              pname.encode(), _comm(mpicomm), algorithm.encode(), options.encode())
        self._register()
        if range is not None:
            range[0], range[1] = rb.value, re.value


class LinearEquations(IterativeSolver):
    def __init__(self, rhs, range=None, aughes=0.0, thresh=1e-10, thresh_value=1e50, hermitian=False, verbosity=0,
                 pname="", mpicomm=None, algorithm="", options=""):
        n = rhs.shape[-1]
        nroot = rhs.shape[0] if rhs.ndim > 1 else 1
        super().__init__(n, nroot)
        rb, re = _range_arrays(range)
        r = np.ascontiguousarray(rhs, dtype=np.float64)
        _call("IterativeSolverLinearEquationsInitialize", n, nroot, C.byref(rb), C.byref(re), _d(r), aughes, thresh,
              thresh_value, 1 if hermitian else 0, verbosity, pname.encode(), _comm(mpicomm), algorithm.encode(),
              options.encode())
        self._register()


class Optimize(IterativeSolver):
    def __init__(self, n, range=None, thresh=1e-10, thresh_value=1e50, verbosity=0, minimize=True, pname="",
                 mpicomm=None, algorithm="", options=""):
        super().__init__(n)
        rb, re = _range_arrays(range)
        _call("IterativeSolverOptimizeInitialize", n, C.byref(rb), C.byref(re), thresh, thresh_value, verbosity,
              1 if minimize else 0, pname.encode(), _comm(mpicomm), algorithm.encode(), options.encode())
        self._register()
