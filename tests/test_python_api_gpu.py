"""The reverse-communication C API (include/iterative_solver_c.h, the reference's
IterativeSolverC.h) and its Python binding (iterative_solver) on the GPU.

* test_diagonalize / test_nonlinear_equations follow the reference's own Python tests
  (python/test/test_rayleigh_quotient.py:101-150) with their assertions (7 decimal places).
* Parity: the C-API loop driven from Python on the dense fixtures takes the same iterations as the
  reference CPU path (oracle.davidson_dense, the restated solve()), eigenvalues within 1e-10.
* P space through IterativeSolverAddP with a caller-side apply-P callback, as the reference's
  examples/LinearEigensystemExampleF-Pspace.F90 drives it (n = 200, 3 roots, 30 P functions).
"""
import json
import os

import numpy as np
import pytest

import iterative_solver
import oracle
from test_python_api import RayleighQuotient

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
BIG = 1.7976931348623157e308


def test_diagonalize():
    problem = RayleighQuotient(8, 0.1)
    nroot = 2
    parameters = np.zeros([nroot, problem.size])
    residual = np.zeros([nroot, problem.size])
    solver = iterative_solver.LinearEigensystem(problem.size, nroot)
    solver.solve(parameters, residual, problem, generate_initial_guess=True)
    solver.solution(list(range(nroot)), parameters, residual)
    assert solver.errors.size == nroot
    for e in solver.errors:
        assert e == pytest.approx(0.0, abs=1e-7)
    ev = solver.eigenvalues
    for root in range(nroot):
        parameters[root] /= np.sqrt(np.dot(parameters[root], parameters[root]))
        value = problem.residual(parameters[root], residual[root])
        assert ev[root] == pytest.approx(problem.eigenvalues[root], abs=1e-7)
        assert value == pytest.approx(ev[root], abs=1e-7)
        assert np.all(np.abs(residual[root]) < 1e-7)
    solver.finalize()


def test_nonlinear_equations():
    problem = RayleighQuotient(4, 0.01)
    parameters = np.zeros(problem.size)
    parameters[0] = 1
    residual = np.zeros(problem.size)
    solver = iterative_solver.NonLinearEquations(problem.size)
    solver.solve(parameters, residual, problem)
    solver.solution([0], parameters, residual)
    parameters = parameters * problem.eigenvectors[0, 0] / parameters[0]
    value = problem.residual(parameters, residual)
    assert value == pytest.approx(problem.eigenvalues[0], abs=1e-7)
    np.testing.assert_allclose(residual, 0.0, atol=1e-7)
    np.testing.assert_allclose(parameters, problem.eigenvectors[:, 0], atol=1e-7)
    solver.finalize()


@pytest.mark.parametrize("algorithm", ["", "SD"])
def test_optimize(algorithm):
    # reference test_rayleigh_quotient.py:76-99 (BFGS is the default algorithm, start x = 10).
    # Plain steepest descent needs a start of unit scale: the Rayleigh gradient scales as 1/|x|.
    problem = RayleighQuotient(4, 0.01)
    parameters = np.full(problem.size, 10.0) if algorithm != "SD" else np.eye(problem.size)[0]
    residual = np.zeros(problem.size)
    solver = iterative_solver.Optimize(problem.size, algorithm=algorithm)
    solver.solve(parameters, residual, problem)
    answer = solver.solution([0], parameters, residual)
    parameters = parameters * problem.eigenvectors[0, 0] / parameters[0]
    assert answer == pytest.approx(problem.eigenvalues[0], abs=1e-7)
    np.testing.assert_allclose(residual, 0.0, atol=1e-7)
    np.testing.assert_allclose(parameters, problem.eigenvectors[:, 0], atol=1e-7)
    solver.finalize()


def check_minimize_flag_ignored():
    # The reference ignores `minimize` (IterativeSolverCMPI.cpp:250-268; its Fortran wrapper may pass
    # an uninitialised value, IterativeSolverF.F90:321, :362-364): minimize=False still minimises.
    problem = RayleighQuotient(4, 0.01)
    parameters = np.full(problem.size, 10.0)
    residual = np.zeros(problem.size)
    solver = iterative_solver.Optimize(problem.size, minimize=False)
    solver.solve(parameters, residual, problem)
    assert solver.solution([0], parameters, residual) == pytest.approx(problem.eigenvalues[0], abs=1e-7)
    solver.finalize()


def test_minimize_flag_ignored():
    check_minimize_flag_ignored()


def check_instance_lifecycle():
    """Each Python solver finalizes its OWN C-layer instance: reassigning a variable in a
    loop creates the new instance before the old object is collected, and the old object's __del__
    must not pop the new one."""
    import gc

    ids = []
    s = None
    for n in (8, 5, 11):
        problem = RayleighQuotient(n, 0.1)
        s = iterative_solver.LinearEigensystem(n, 1)  # the previous s dies here, after the new push
        gc.collect()
        ids.append(s._id)
        x, g = np.zeros([1, n]), np.zeros([1, n])
        s.solve(x, g, problem, generate_initial_guess=True)
        assert s.eigenvalues[0] == pytest.approx(problem.eigenvalues[0], abs=1e-7)
    assert len(set(ids)) == 3
    # an older live object must not drive the newer instance
    t = iterative_solver.LinearEigensystem(6, 1)
    with pytest.raises(RuntimeError, match="another IterativeSolver instance is active"):
        s.errors
    t.finalize()
    assert s.errors.size == 1  # s is the top again
    s.finalize()
    with pytest.raises(RuntimeError, match="finalized"):
        s.errors
    del s, t
    gc.collect()


def test_instance_lifecycle():
    check_instance_lifecycle()


def test_linear_equations():
    # reference test_rayleigh_quotient.py:152-181
    problem = RayleighQuotient(33, 0.1)
    nroot = 2
    parameters = np.zeros([nroot, problem.size])
    residual = np.zeros([nroot, problem.size])
    rhs = np.array([problem.eigenvalues[r] * problem.eigenvectors[:, r] for r in range(nroot)])
    solver = iterative_solver.LinearEquations(rhs=rhs, thresh=1e-9)
    solver.solve(parameters, residual, problem, generate_initial_guess=True)
    solver.solution(list(range(nroot)), parameters, residual)
    assert solver.errors.size == nroot
    assert np.all(np.abs(solver.errors) < 1e-7)
    for root in range(nroot):
        v = problem.eigenvectors[0, root] * parameters[root] / parameters[root, 0]
        np.testing.assert_allclose(v, problem.eigenvectors[:, root], atol=1e-7)
        np.testing.assert_allclose(residual[root], 0.0, atol=1e-7)
    solver.finalize()


def test_simple_linear_equations():
    # reference test_rayleigh_quotient.py:183-215: M_ij = i + j + 1 (+1 diagonal), x_r = r + 1
    class Simple(RayleighQuotient):
        @property
        def matrix(self):
            return np.add.outer(np.arange(self.size), np.arange(self.size)) + 1.0 + np.eye(self.size)

    problem = Simple(8)
    nroot = 2
    parameters = np.zeros([nroot, 8])
    residual = np.zeros([nroot, 8])
    rhs = np.array([[(r + 1) * (8 * 9 / 2 + i * 8 + 1) for i in range(8)] for r in range(nroot)])
    solver = iterative_solver.LinearEquations(rhs=rhs)
    solver.solve(parameters, residual, problem, generate_initial_guess=True)
    solver.solution(list(range(nroot)), parameters, residual)
    assert np.all(np.abs(solver.errors) < 1e-7)
    np.testing.assert_allclose(parameters, np.outer([1.0, 2.0], np.ones(8)), atol=1e-7)
    np.testing.assert_allclose(residual, 0.0, atol=1e-7)
    solver.finalize()


class Dense(iterative_solver.Problem):
    """Dense symmetric H with the C++ default preconditioner a / ((d - shift) + 1e-15)
    (reference IterativeSolver.h:47-55), as the oracle's dense problem uses."""

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


def hamiltonian(name, split):
    t = open(os.path.join(GOLD, name + ".hamiltonian")).read().split()
    n = int(t[0])
    return np.array(t[1:1 + n * n], dtype=float).reshape(n, n) + np.diag(split * np.arange(n))


@pytest.mark.parametrize("name,split,nroot", [("he", 0.0, 1), ("hf", 1e-8, 1), ("hf", 1e-8, 3), ("bh", 1e-8, 1),
                                              ("bh", 1e-8, 3)])
def test_c_api_loop_matches_reference_path(name, split, nroot):
    h = hamiltonian(name, split)
    n = h.shape[0]
    kw = dict(nroots=nroot, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
    cpu = oracle.davidson_dense(h, **kw)
    solver = iterative_solver.LinearEigensystem(n, nroot, thresh=1e-8, thresh_value=BIG, hermitian=True,
                                                options=f"MAX_SIZE_QSPACE={6 * nroot},RESET_D=8")
    x, g = np.zeros((nroot, n)), np.zeros((nroot, n))
    # the C++ solve()'s initial guess: unit vectors on the nroot smallest diagonals, in index order
    for k, i in enumerate(sorted(np.argsort(np.diag(h), kind="stable")[:nroot])):
        x[k, i] = 1.0
    solver.solve(x, g, Dense(h))
    st = solver.statistics()
    assert st["iterations"] == cpu["iterations"]
    ev = solver.eigenvalues
    assert np.max(np.abs(ev - cpu["eigenvalues"])) <= 1e-10 * max(1.0, np.max(np.abs(cpu["eigenvalues"])))
    gold = json.load(open(os.path.join(GOLD, "eigen_golden.json")))[name]["eigenvalues"][:nroot]
    assert np.max(np.abs(ev - np.array(gold))) < 1e-10
    assert np.all(solver.errors <= 2e-8)
    solver.finalize()


def test_add_p_with_caller_callback():
    # reference examples/LinearEigensystemExampleF-Pspace.F90: m = 1 + diag(3 i), P = first 30 unit vectors
    n, nroot, nP = 200, 3, 30
    m = np.ones((n, n)) + np.diag(3.0 * np.arange(1, n + 1))
    pidx = np.arange(nP)
    solver = iterative_solver.LinearEigensystem(n, nroot, thresh=1e-8, thresh_value=BIG, hermitian=True)
    c, g = np.zeros((nroot, n)), np.zeros((nroot, n))
    calls = []

    def apply_p(pc, gl, ranges):
        calls.append(pc.shape[0])
        for k in range(pc.shape[0]):
            r0, r1 = ranges[k]
            gl[k * n:k * n + (r1 - r0)] += m[r0:r1][:, pidx] @ pc[k]

    nwork = solver.add_p([{int(i): 1.0} for i in pidx], m[np.ix_(pidx, pidx)], c, g, apply_p)
    d = np.diag(m)
    for _ in range(100):
        ev = solver.working_set_eigenvalues(nwork)
        for k in range(nwork):
            g[k] = g[k] / ((d - ev[k]) + 1e-15)
        nwork = solver.end_iteration(c, g)
        if nwork == 0:
            break
        g[:nwork] = c[:nwork] @ m
        nwork = solver.add_vector(c[:nwork], g[:nwork])
        if nwork == 0:
            break
    assert nwork == 0 and calls
    np.testing.assert_allclose(solver.eigenvalues, np.linalg.eigvalsh(m)[:nroot], rtol=0, atol=1e-8)
    assert np.all(solver.errors <= 1e-8)
    solver.finalize()


def check_factory_dispatch():
    rhs = np.ones((1, 4))
    bad = [
        lambda: iterative_solver.LinearEigensystem(4, 1, algorithm="Lanczos"),
        lambda: iterative_solver.LinearEquations(rhs, algorithm="CG"),
        lambda: iterative_solver.NonLinearEquations(4, algorithm="Newton"),
        lambda: iterative_solver.Optimize(4, algorithm="LBFGS"),
    ]
    for make in bad:
        try:
            make()
        except RuntimeError as e:
            assert "Unimplemented method" in str(e), str(e)
        else:
            raise AssertionError("unknown method accepted")
    for make in (
        lambda: iterative_solver.LinearEigensystem(4, 1, algorithm="Davidson"),
        lambda: iterative_solver.LinearEigensystem(4, 1, algorithm="RSPT", options="max_iter=5"),
        lambda: iterative_solver.LinearEquations(rhs, algorithm="Davidson"),
        lambda: iterative_solver.NonLinearEquations(4, algorithm="DIIS"),
        lambda: iterative_solver.Optimize(4, algorithm="SD"),
        lambda: iterative_solver.Optimize(4, algorithm=""),
    ):
        make().finalize()


def test_solver_factory_dispatch():
    # C API method names through the SolverFactory restatement (reference SolverFactory.h:114-185):
    # unknown methods raise "Unimplemented method <m>"; Davidson/RSPT/DIIS/BFGS/SD construct
    check_factory_dispatch()


def test_python_api_is_the_cpu_path_bit_for_bit(tmp_path):
    """The reference's Python tests and the dense C-API loops (tests/api_cases.py) on the HIP path
    against the CPU path -- the same host code over the host emulation of the device ABI, in a process
    of its own (tests/emul_worker.py api_record) -- every eigenvalue, error, solution and residual
    element and every iteration count bit for bit: at these sizes the HIP path computes in the
    reference's arithmetic (ssp_ctx_set_exact_max)."""
    import subprocess
    import sys

    import api_cases

    out = tmp_path / "api_emul.json"
    worker = os.path.join(os.path.dirname(__file__), "emul_worker.py")
    subprocess.run([sys.executable, worker, "api_record", str(out)], check=True, timeout=600, capture_output=True)
    cpu = json.load(open(out))
    gpu = json.loads(json.dumps(api_cases.run_all(iterative_solver)))
    assert gpu.keys() == cpu.keys()
    for key in cpu:
        for field, value in cpu[key].items():
            assert np.array_equal(np.asarray(gpu[key][field]), np.asarray(value)), (key, field)
