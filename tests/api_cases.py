"""The reference's Python tests (python/test/test_rayleigh_quotient.py) and the C-API loop on the dense
fixtures, as one function that runs them through whichever `iterative_solver` library is loaded and
returns every result (eigenvalues, errors, solutions, values, iteration counts).  TEST INFRASTRUCTURE:
tests/test_python_api_gpu.py runs it on the HIP path in process and through tests/emul_worker.py
(`api_record`) on the CPU path -- the same host code over the host emulation of the device ABI, in
the reference's arithmetic -- and compares the two bit for bit.
"""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BIG = 1.7976931348623157e308


def hamiltonian(name, split):
    t = open(os.path.join(GOLD, name + ".hamiltonian")).read().split()
    n = int(t[0])
    return np.array(t[1:1 + n * n], dtype=float).reshape(n, n) + np.diag(split * np.arange(n))


def run_all(iterative_solver):
    from test_python_api import RayleighQuotient

    class Dense(iterative_solver.Problem):
        def __init__(self, h):
            super().__init__()
            self.h = h

        def action(self, parameters, actions):
            np.matmul(parameters, self.h, out=actions)

        def diagonals(self, d):
            d[: self.h.shape[0]] = np.diag(self.h)
            return True

        def precondition(self, residual, shift=None, diagonals=None):
            for i in range(residual.shape[0]):
                residual[i] = residual[i] / ((diagonals - shift[i]) + 1e-15)

    out = {}

    def record(key, solver, parameters, residual, extra=None):
        out[key] = {"errors": np.asarray(solver.errors).tolist(), "parameters": np.asarray(parameters).tolist(),
                    "residual": np.asarray(residual).tolist(), "iterations": solver.statistics()["iterations"],
                    **(extra or {})}

    # test_rayleigh_quotient.py:101-128 diagonalize
    problem = RayleighQuotient(8, 0.1)
    x, g = np.zeros([2, 8]), np.zeros([2, 8])
    s = iterative_solver.LinearEigensystem(8, 2)
    s.solve(x, g, problem, generate_initial_guess=True)
    s.solution([0, 1], x, g)
    record("diagonalize", s, x, g, {"eigenvalues": np.asarray(s.eigenvalues).tolist()})
    s.finalize()
    # :130-150 nonlinear equations
    problem = RayleighQuotient(4, 0.01)
    x, g = np.zeros(4), np.zeros(4)
    x[0] = 1
    s = iterative_solver.NonLinearEquations(4)
    s.solve(x, g, problem)
    s.solution([0], x, g)
    record("nonlinear_equations", s, x, g)
    s.finalize()
    # :76-99 optimize (BFGS from x = 10; SD from e_0)
    for alg in ("", "SD"):
        problem = RayleighQuotient(4, 0.01)
        x = np.full(4, 10.0) if alg != "SD" else np.eye(4)[0]
        g = np.zeros(4)
        s = iterative_solver.Optimize(4, algorithm=alg)
        s.solve(x, g, problem)
        value = s.solution([0], x, g)
        record(f"optimize/{alg or 'BFGS'}", s, x, g, {"value": float(value)})
        s.finalize()
    # :152-181 linear equations
    problem = RayleighQuotient(33, 0.1)
    rhs = np.array([problem.eigenvalues[r] * problem.eigenvectors[:, r] for r in range(2)])
    x, g = np.zeros([2, 33]), np.zeros([2, 33])
    s = iterative_solver.LinearEquations(rhs=rhs, thresh=1e-9)
    s.solve(x, g, problem, generate_initial_guess=True)
    s.solution([0, 1], x, g)
    record("linear_equations", s, x, g)
    s.finalize()
    # the C-API loop on the dense fixtures
    for name, split, nroot in (("he", 0.0, 1), ("hf", 1e-8, 1), ("hf", 1e-8, 3), ("bh", 1e-8, 1), ("bh", 1e-8, 3)):
        h = hamiltonian(name, split)
        n = h.shape[0]
        s = iterative_solver.LinearEigensystem(n, nroot, thresh=1e-8, thresh_value=BIG, hermitian=True,
                                               options=f"MAX_SIZE_QSPACE={6 * nroot},RESET_D=8")
        x, g = np.zeros((nroot, n)), np.zeros((nroot, n))
        for k, i in enumerate(sorted(np.argsort(np.diag(h), kind="stable")[:nroot])):
            x[k, i] = 1.0
        s.solve(x, g, Dense(h))
        record(f"dense/{name}/{nroot}", s, x, g, {"eigenvalues": np.asarray(s.eigenvalues).tolist()})
        s.finalize()
    return out
