"""The reference's Python API (python/iterative_solver) on the HBM back end: import and Problem
semantics here (CPU), the solver runs in tests/test_python_api_gpu.py.  The Rayleigh-quotient
problem and its assertions follow the reference's python/test/test_rayleigh_quotient.py."""
import numpy as np
import pytest

import iterative_solver


class RayleighQuotient(iterative_solver.Problem):
    """M_ij = (i+1) delta_ij + rho; f(x) = x.Mx / x.x (reference test_rayleigh_quotient.py:8-50)."""

    def __init__(self, n, rho=0.1):
        super().__init__()
        self.size = n
        self.rho = rho

    @property
    def matrix(self):
        return self.rho * np.ones((self.size, self.size)) + np.diag(np.arange(1.0, self.size + 1))

    def residual(self, parameters, gradient):
        self.action(parameters.reshape([1, parameters.size]), gradient.reshape([1, parameters.size]))
        xx = np.dot(parameters, parameters)
        f = np.dot(parameters, gradient) / xx
        gradient[:] = 2 * (gradient - f * parameters) / xx
        return f

    def action(self, parameters, residual):
        np.matmul(parameters, self.matrix, out=residual)

    def diagonals(self, diagonals):
        diagonals[: self.size] = np.diag(self.matrix)
        return True

    @property
    def eigenvalues(self):
        return np.linalg.eigh(self.matrix)[0]

    @property
    def eigenvectors(self):
        return np.linalg.eigh(self.matrix)[1]


def test_problem_gradient_is_exact():
    # reference test_rayleigh_quotient.py:61-74
    problem = RayleighQuotient(4, 0.01)
    parameters = np.ones(problem.size) * 77
    residual = np.zeros(problem.size)
    step = 1e-5
    parameters[0] += step
    f1 = problem.residual(parameters, residual)
    parameters[0] -= 2 * step
    fm1 = problem.residual(parameters, residual)
    parameters[0] += step
    problem.residual(parameters, residual)
    assert (f1 - fm1) / (2 * step) == pytest.approx(residual[0], abs=1e-7)


def test_default_preconditioner_matches_reference_formula():
    # reference problem.py:69-80: r_j / (d_j + shift + 1e-14), row by row
    p = iterative_solver.Problem()
    r = np.array([[1.0, -2.0, 3.0], [0.5, 0.25, -1.0]])
    d = np.array([1.0, 2.0, 4.0])
    shift = np.array([0.5, -0.25])
    want = np.array([[r[i, j] / (d[j] + shift[i] + 1e-14) for j in range(3)] for i in range(2)])
    p.precondition(r, shift=shift, diagonals=d)
    assert np.array_equal(r, want)


def test_classes_mirror_reference_api():
    for name in ("Problem", "IterativeSolver", "LinearEigensystem", "NonLinearEquations", "LinearEquations",
                 "Optimize"):
        assert hasattr(iterative_solver, name)
    for meth in ("solve", "solution", "add_vector", "end_iteration", "add_value", "add_p", "mpicomm_compute"):
        assert callable(getattr(iterative_solver.IterativeSolver, meth))
    assert isinstance(iterative_solver.LinearEigensystem.eigenvalues, property)
    assert isinstance(iterative_solver.IterativeSolver.errors, property)
