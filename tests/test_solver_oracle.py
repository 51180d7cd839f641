"""Pins the reference CPU solver path (oracle/itsolv_oracle.cpp: restated Davidson / DIIS over the
oracle's ArrayHandlerIterable restatement) against golden eigenvalues computed independently
(tests/golden/make_golden.py) and the reference tests' own assertions:
  errors <= 2 * threshold, eigenvalues within 2e-9 / 1e-10 of the full diagonalisation,
  r_creations <= (nroot + 1) * n_iter   (reference test/itsolv/test_LinearEigensystem.cpp:300-341)
  DIIS: x -> 1 within threshold          (reference test/itsolv/test_NonLinearEquations.cpp:105-106)
"""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
G = json.load(open(os.path.join(GOLD, "eigen_golden.json")))


def hamiltonian(name, split):
    t = open(os.path.join(GOLD, name + ".hamiltonian")).read().split()
    n = int(t[0])
    return np.array(t[1 : 1 + n * n], dtype=float).reshape(n, n) + np.diag(split * np.arange(n))


def check_reference_invariants(r, nroot, thresh=1e-8):
    assert r["converged"]
    assert np.all(r["errors"] <= 2 * thresh)
    assert r["r_creations"] <= (nroot + 1) * (r["iterations"] + 2)
    assert np.all(r["residual_norms"] <= 10 * thresh)


@pytest.mark.parametrize("name,split", [("he", 0.0), ("hf", 1e-8), ("bh", 1e-8)])
@pytest.mark.parametrize("nroot", [1, 2, 3])
@pytest.mark.parametrize("np_", [0, 4])
def test_fixture_eigenvalues(name, split, nroot, np_):
    h = hamiltonian(name, split)
    n = h.shape[0]
    if name == "he" and nroot > 1:
        pytest.skip("he has a degenerate pair: eigenvectors ill-defined (reference splits only bh/hf)")
    if np_ and np_ < nroot:
        np_ = nroot
    r = oracle.davidson_dense(h, nroots=nroot, max_p=min(np_, n), convergence_threshold=1e-8,
                              max_size_qspace=max(6 * nroot, min(n, 6 * nroot) - np_), reset_D=8)
    check_reference_invariants(r, nroot)
    ref = np.array(G[name]["eigenvalues"][:nroot])
    assert np.max(np.abs(r["eigenvalues"] - ref)) < 1e-10
    if name == "he":
        # FCI energy from reference examples/he.molpro/run/5.molpro/5.out:408 (Hamiltonian file has 9 digits)
        assert abs(r["eigenvalues"][0] - G["he"]["fci_energy"]) < 1e-8


def test_ones_matrix_100_with_pspace():
    # reference test_LinearEigensystem.cpp:41-51, n = 100, param = 1; P space of 20
    n = 100
    h = np.ones((n, n)) + np.diag(np.arange(n) - 1.0)
    for nroot, np_ in ((1, 0), (3, 20), (5, 20)):
        r = oracle.davidson_dense(h, nroots=nroot, max_p=np_, convergence_threshold=1e-8, max_size_qspace=6 * nroot,
                                  reset_D=8)
        check_reference_invariants(r, nroot)
        assert np.max(np.abs(r["eigenvalues"] - np.array(G["ones_100"]["eigenvalues"][:nroot]))) < 2e-9


def test_rayleigh_quotient_4():
    # reference test_rayleigh_quotient.cpp:157-170 (Davidson, threshold 1e-10)
    g = G["rayleigh_4"]
    h = np.full((4, 4), g["rho"]) + np.diag(np.arange(4) + 1.0)
    r = oracle.davidson_dense(h, nroots=1, convergence_threshold=1e-10)
    assert r["converged"]
    assert abs(r["eigenvalues"][0] - g["eigenvalues"][0]) < 1e-10
    v = r["solutions"][0] / np.linalg.norm(r["solutions"][0])
    np.testing.assert_allclose(np.abs(v), g["lowest_eigenvector_abs"], atol=1e-9)


@pytest.mark.parametrize("n", [2, 3, 7, 20, 50])
def test_diis_quadratic_form(n):
    # reference test_NonLinearEquations.cpp:25-31, :62-121: H = 1 + diag((i + 2) * 10), x -> 1
    h = np.ones((n, n)) + np.diag((np.arange(n) + 2) * 10.0)
    r = oracle.diis_dense(h, convergence_threshold=1e-8, max_size_qspace=6)
    assert r["converged"]
    assert r["errors"][0] <= 2e-8
    assert r["r_creations"] <= 2 * (r["iterations"] + 1)
    np.testing.assert_allclose(r["x"], np.ones(n), atol=1e-8)


@pytest.mark.parametrize("nroot", [1, 4])
def test_rank_one_synthetic_secular_equation(nroot):
    n, rho = 3000, 0.1
    r = oracle.davidson_synthetic(n, rho, 1, 1, nroots=nroot, convergence_threshold=1e-9, max_size_qspace=6 * nroot,
                                  reset_D=8)
    assert r["converged"]
    np.testing.assert_allclose(r["eigenvalues"], oracle.rank_one_eigenvalues(n, rho, nroot), rtol=1e-12, atol=0)


def test_rank_r_synthetic_dense_reference():
    n, rho, rank, seed = 800, 0.1, 4, 5
    u = oracle.synthetic_signs(n, rank, seed)
    h = np.diag(1.0 + np.arange(n)) + rho * u.T @ u
    ref = np.linalg.eigvalsh(h)[:6]
    for np_ in (0, 8):
        r = oracle.davidson_synthetic(n, rho, rank, seed, nroots=6, max_p=np_, convergence_threshold=1e-9,
                                      max_size_qspace=24, reset_D=8)
        assert r["converged"]
        assert np.max(np.abs(r["eigenvalues"] - ref)) < 1e-10


def nonhermitian_matrix(n, param, non_hermiticity):
    # reference test_LinearEigensystem.cpp:40-50: H = 1, H_ii = i*param, lower triangle *(1 - nh)
    h = np.ones((n, n))
    h[np.diag_indices(n)] = np.arange(n) * param
    h[np.tril_indices(n, -1)] *= 1 - non_hermiticity
    return h


@pytest.mark.parametrize("param", [1.0, 0.1])
@pytest.mark.parametrize("nh", [0.0, 0.1, 0.2])
@pytest.mark.parametrize("nroot", [1, 2, 3])
def test_nonhermitian_eigen(param, nh, nroot):
    # reference test_LinearEigensystem.cpp:364-375 (n = 6), checked against numpy's general eigensolver
    h = nonhermitian_matrix(6, param, nh)
    r = oracle.davidson_dense(h, nroots=nroot, hermitian=0, convergence_threshold=1e-9)
    assert r["converged"]
    exact = np.sort(np.linalg.eigvals(h).real)[:nroot]
    assert np.max(np.abs(r["eigenvalues"] - exact)) < 1e-10


def simple_system(n, nroot):
    # reference test_LinearEquations.cpp:17-38: A_ij = i + j + 1 (+1 on the diagonal), x_r = r + 1
    a = np.add.outer(np.arange(n), np.arange(n)) + 1.0 + np.eye(n)
    rhs = np.array([[(r + 1) * (n * (n + 1) / 2 + j * n + 1) for j in range(n)] for r in range(nroot)])
    return a, rhs


@pytest.mark.parametrize("n", [3, 6, 12, 21, 33])
@pytest.mark.parametrize("nroot", [1, 2, 3, 13])
def test_linear_equations_symmetric_system(n, nroot):
    # reference test_LinearEquations.cpp:59-99 (threshold 1e-10, solution to 1e-5)
    if nroot > n:
        pytest.skip("more roots than the dimension")
    a, rhs = simple_system(n, nroot)
    r = oracle.linear_equations_dense(a, rhs, nroots=nroot, convergence_threshold=1e-10)
    assert r["converged"]
    np.testing.assert_allclose(r["x"], np.outer(np.arange(1, nroot + 1), np.ones(n)), atol=1e-5, rtol=0)
    assert np.all(r["residual_norms"][:nroot] <= 1e-9)


@pytest.mark.parametrize("aug", [0.5, 1.0])
def test_linear_equations_augmented_hessian_subspace_solve(aug):
    # Augmented Hessian (reference helper-implementation.h:561-594): the subspace solution is
    # x = (A - e)^-1 b with e the lowest eigenvalue of [[A, -a b], [-a b^T, 0]].  Once the subspace
    # spans the whole space (n = 4) that is the full-space value; the residual A x - b then stays
    # e x, so the run ends unconverged when no new direction remains.
    n = 4
    a = np.full((n, n), 0.1) + np.diag(np.arange(1.0, n + 1))
    rhs = np.sin(np.arange(n) + 1.0)[None, :]
    r = oracle.linear_equations_dense(a, rhs, nroots=1, convergence_threshold=1e-10, augmented_hessian=aug, max_iter=20)
    m = np.block([[a, -aug * rhs.T], [-aug * rhs, np.zeros((1, 1))]])
    e = np.linalg.eigvalsh(m)[0]
    np.testing.assert_allclose(r["x"][0], np.linalg.solve(a - e * np.eye(n), rhs[0]), atol=1e-12)


def rayleigh_matrix(n, rho):
    # reference python/test/test_rayleigh_quotient.py:16-22: M_ij = (i + 1) delta_ij + rho
    return np.full((n, n), rho) + np.diag(np.arange(1.0, n + 1))


@pytest.mark.parametrize("n,alg,thresh", [(4, "BFGS", 1e-8), (20, "BFGS", 1e-6), (100, "BFGS", 1e-6),
                                          (4, "SD", 1e-8), (20, "SD", 1e-6)])
def test_optimize_rayleigh_quotient(n, alg, thresh):
    # OptimizeBFGS / OptimizeSD minimising x.Mx / x.x from e_0: the value is the lowest eigenvalue
    m = rayleigh_matrix(n, 0.01)
    r = oracle.optimize_dense(m, alg, convergence_threshold=thresh, max_iter=200)
    assert r["converged"]
    assert abs(r["eigenvalues"][0] - np.linalg.eigvalsh(m)[0]) < 1e-12
    assert r["residual_norms"][0] <= thresh


# Option block_gram_schmidt (extension, itsolv_options.block_gram_schmidt): the MGS projection from
# the overlaps append_overlap_with_r already holds + one gemm_outer per space.  Its own parity
# sign-off against the reference's sequential sweep: the same iterations and
# eigenvalues within 1e-10 on the reference fixtures, P space included, and on synthetic problems.
@pytest.mark.parametrize("name,split,nroot,np_", [("he", 0.0, 1, 0), ("hf", 1e-8, 1, 0), ("hf", 1e-8, 3, 0),
                                                  ("bh", 1e-8, 1, 0), ("bh", 1e-8, 3, 0), ("bh", 1e-8, 6, 0),
                                                  ("bh", 1e-8, 3, 6), ("hf", 1e-8, 1, 4)])
def test_block_gram_schmidt_matches_sequential_fixtures(name, split, nroot, np_):
    h = hamiltonian(name, split)
    kw = dict(nroots=nroot, max_p=np_, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
    ref, blk = oracle.davidson_dense(h, **kw), oracle.davidson_dense(h, block_gram_schmidt=1, **kw)
    assert blk["converged"] and blk["iterations"] == ref["iterations"] and blk["r_creations"] == ref["r_creations"]
    np.testing.assert_allclose(blk["eigenvalues"], ref["eigenvalues"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("n,rank,rho,nroot,maxq,np_", [(1000, 1, 0.1, 1, 6, 0), (1000, 4, 0.1, 4, 24, 0),
                                                       (20_000, 8, 0.1, 8, 48, 0), (20_000, 8, 0.1, 8, 48, 16),
                                                       (50_000, 3, 0.01, 2, 12, 8)])
def test_block_gram_schmidt_matches_sequential_synthetic(n, rank, rho, nroot, maxq, np_):
    kw = dict(nroots=nroot, convergence_threshold=1e-8, max_size_qspace=maxq, reset_D=8, max_p=np_)
    ref = oracle.davidson_synthetic(n, rho, rank, 1, **kw)
    blk = oracle.davidson_synthetic(n, rho, rank, 1, block_gram_schmidt=1, **kw)
    assert blk["converged"] and blk["iterations"] == ref["iterations"]
    np.testing.assert_allclose(blk["eigenvalues"], ref["eigenvalues"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("n,nroot", [(12, 3), (33, 2)])
def test_block_gram_schmidt_linear_equations(n, nroot):
    a, rhs = simple_system(n, nroot)
    kw = dict(nroots=nroot, convergence_threshold=1e-10)
    ref = oracle.linear_equations_dense(a, rhs, **kw)
    blk = oracle.linear_equations_dense(a, rhs, block_gram_schmidt=1, **kw)
    assert blk["converged"] and blk["iterations"] == ref["iterations"]
    np.testing.assert_allclose(blk["x"], ref["x"], atol=2e-6, rtol=0)


def test_interpolate_cubic_constructor():
    # reference test/itsolv/test_Interpolate.cpp:7-21: f = x (x - 1/2)^2 through (0, 0, 1/4), (1, 1/4, 5/4)
    p0, p1 = (0.0, 0.0, 0.25), (1.0, 0.25, 1.25)
    assert oracle.interpolate_cubic(p0, p1, 0.0).tolist() == [0.0, 0.0, 0.25, -2.0]
    assert oracle.interpolate_cubic(p0, p1, 1.0).tolist() == [1.0, 0.25, 1.25, 4.0]
    assert oracle.interpolate_cubic(p0, p1, 0.5)[2] == 0.0


def test_interpolate_cubic_minimum():
    # test_Interpolate.cpp:23-41 with the analytic cubic minimiser OptimizeBFGS uses
    # (OptimizeBFGS.h:95-96; Interpolate.cpp:141-142)
    p = oracle.interpolate_minimize((0.0, 0.0, 0.25), (1.0, 0.25, 1.25), 0.0, 1.0)
    assert abs(p[0] - 0.5) < 1e-13 and abs(p[1]) < 1e-13 and abs(p[2]) < 1e-13 and p[3] > 0


def test_interpolate_minimize_bracketing():
    # test_Interpolate.cpp:23-41 (Interpolate.minimize): the grid-bracketing + regula-falsi search
    # (analytic = false) on f = x (x - 1/2)^2, every assertion of the reference test
    p0, p1 = (0.0, 0.0, 0.25), (1.0, 0.25, 1.25)

    def mini(xa, xb, grid=100, grid_max=100000):
        return oracle.interpolate(p0, p1, "cubic", xa=xa, xb=xb, bracket_grid=grid, max_bracket_grid=grid_max,
                                  analytic=False)[1]

    assert abs(mini(0, 1, 5, 1000)[0] - 0.5) < 1e-13
    assert abs(mini(0, 1)[1]) < 1e-13
    assert abs(mini(0, 1)[2]) < 1e-13
    assert mini(0.3, 0.6)[3] > 0
    assert abs(mini(0, -1)[0] + 1) < 1e-13
    assert abs(mini(0.51, 1)[0] - 0.51) < 1e-13
    assert abs(mini(0.1, 2)[0] - 0.5) < 1e-13
    assert abs(mini(-1200, 2)[0] - 0.5) < 1e-13
    assert abs(mini(0.4, 200)[0] - 0.5) < 1e-13


@pytest.mark.parametrize("interpolant", ["cubic", "morse"])
def test_interpolate_quadratic(interpolant):
    # test_Interpolate.cpp:43-58: f = (x - 1/2)^2 + lambda x^3 through (0, 1/4, -1), (1, 1/4 + l, 1 + 3l);
    # both interpolants' minimum on [0, 1] is the exact one to 1e-8
    lam = 1e-3
    p0, p1 = (0.0, 0.25, -1.0), (1.0, 0.25 + lam, 1 + 3 * lam)
    at0, m, par = oracle.interpolate(p0, p1, interpolant, x=0.0, xa=0.0, xb=1.0)
    x_expected = (-2.0 + np.sqrt(4.0 + 12 * lam)) / (6 * lam)
    assert abs(m[0] - x_expected) < 1e-8
    # the interpolant reproduces the defining values and slopes (the Morse fit's DIIS residual)
    at1 = oracle.interpolate(p0, p1, interpolant, x=1.0)[0]
    np.testing.assert_allclose([at0[1], at0[2], at1[1], at1[2]], [p0[1], p0[2], p1[1], p1[2]], atol=1e-9)
    if interpolant == "morse":
        # L0 + (k / 2a^2)(1 - exp(-a (y - y0)))^2: minimum L0 at y0
        assert abs(m[0] - par[3]) < 1e-8 and abs(m[1] - par[0]) < 1e-12


def test_interpolate_unknown():
    with pytest.raises(RuntimeError, match="Unknown interpolant: spline"):
        oracle.interpolate((0.0, 0.0, 0.25), (1.0, 0.25, 1.25), "spline")


@pytest.mark.parametrize("n", [1, 2])
def test_test_problem_trig(n):
    # reference test_NonLinearEquations.cpp:206-213: test_problem accepts trigProblem at 1e-9 ...
    assert oracle.itsolv_lib().oracle_test_problem_trig(n, 1e-9, 0) == 1
    # ... and rejects the same problem with a residual 10 % too large
    assert oracle.itsolv_lib().oracle_test_problem_trig(n, 1e-9, 1) == 0
