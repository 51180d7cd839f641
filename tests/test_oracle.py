"""Pins the oracle (oracle/oracle_ops.c) against the reference's own known answers and against
golden vectors computed independently with numpy (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLDEN, "ops_golden.npz"))


def test_select_max_dot_known_answer():
    # reference test/array/testArrayHandlerIterable.cpp:64-68
    x = [1, -2, 1, 0, 3, 0, -4, 1]
    y = [1, 1, 1, 1, 1, 1, 1, 1]
    idx, val = oracle.select_max_dot(x, y, 3)
    assert dict(zip(idx.tolist(), val.tolist())) == {6: 4.0, 4: 3.0, 1: 2.0}


def test_sparse_dot_known_answer():
    # reference test/array/testArrayHandlerIterableSparse.cpp:22-29
    x = [1, 1.0, 1, 2.0, 1, 3.0, 0, 1, 1, 1, 1, 4.0]
    y = {1: 1.0, 3: 2.0, 6: 3.0, 11: 4.0}
    assert oracle.sparse_dot(x, list(y), list(y.values())) == 1.0 + 2.0 * 2.0 + 4.0 * 4.0


def test_gemm_inner_equals_pairwise_dot():
    # reference test/array/testGemm.cpp:58-88 (iota vectors, DoubleEq)
    n = dim = 10
    vx = [np.arange(dim) + i + 0.5 for i in range(n)]
    vy = [np.arange(dim) + i + 0.5 for i in range(n)]
    gemm = oracle.gemm_inner(vx, vy)
    ref = np.array([[oracle.dot(a, b) for b in vy] for a in vx])
    assert np.array_equal(gemm, ref)


def test_dot_axpy_sizes_follow_reference_errors():
    # ArrayHandlerIterable.h:68-69, :77-78
    with pytest.raises(oracle.OracleError):
        oracle.dot(np.ones(3), np.ones(2))
    with pytest.raises(oracle.OracleError):
        oracle.axpy(1.0, np.ones(2), np.ones(3))
    with pytest.raises(oracle.OracleError):
        oracle.select(np.ones(3), 4)


def test_ops_against_golden(g):
    xs, ys = list(g["xs"]), list(g["ys"])
    np.testing.assert_allclose(oracle.gemm_inner(xs, ys), g["gemm_inner"], rtol=1e-13, atol=1e-12)
    out = oracle.gemm_outer(g["alphas"], ys, xs)
    np.testing.assert_allclose(np.array(out), g["gemm_outer"], rtol=1e-13, atol=1e-13)
    pre = oracle.precondition(xs, g["diag"], g["shift"])
    np.testing.assert_array_equal(np.array(pre), g["precondition"])  # same IEEE ops, same order


def test_select_tie_rule_against_golden(g):
    sel = g["sel"]
    idx, val = oracle.select(sel, 9)
    assert idx.tolist() == g["select_min_idx"].tolist()
    assert np.array_equal(val, sel[idx])
    idx, val = oracle.select(sel, 9, max=True, ignore_sign=True)
    assert idx.tolist() == g["select_max_abs_idx"].tolist()
    assert np.array_equal(val, np.abs(sel[idx]))


def test_select_prefers_larger_index_on_ties():
    idx, val = oracle.select(np.array([1.0, 0.0, 0.0, 0.0, 2.0]), 2)
    assert idx.tolist() == [2, 3]


def test_sparse_ops():
    n = 12
    idx = [1, 3, 6, 11]
    val = [1.0, 2.0, 3.0, 4.0]
    x = oracle.sparse_copy(n, idx, val)
    assert x.tolist() == [0, 1, 0, 2, 0, 0, 3, 0, 0, 0, 0, 4]
    y = oracle.sparse_axpy(2.0, idx + [20], val + [9.0], np.ones(n))  # index >= size is skipped
    assert y[11] == 9.0 and y[0] == 1.0


@pytest.mark.parametrize("dim,chunks", [(10, 3), (100000000, 8), (7, 8), (0, 2)])
def test_distribution_spread_remainder(dim, chunks):
    b = oracle.distribution(dim, chunks)
    sizes = np.diff(b)
    assert b[0] == 0 and b[-1] == dim
    extra = dim % chunks
    assert all(s == dim // chunks + (1 if c < extra else 0) for c, s in enumerate(sizes))


def test_rank_one_secular_equation_matches_dense():
    n, rho = 50, 0.1
    h = np.diag(1.0 + np.arange(n)) + rho
    ref = np.linalg.eigvalsh(h)[:5]
    np.testing.assert_allclose(oracle.rank_one_eigenvalues(n, rho, 5), ref, rtol=1e-13)


def test_synthetic_problem_restatement():
    n, rho, rank, seed = 64, 0.1, 3, 7
    u = oracle.synthetic_signs(n, rank, seed)
    h = np.diag(1.0 + np.arange(n)) + rho * u.T @ u
    x = oracle.random_vector(n, seed, 3)
    np.testing.assert_allclose(oracle.synthetic_action(x, rho, rank, seed), h @ x, rtol=1e-13, atol=1e-13)
    np.testing.assert_array_equal(oracle.synthetic_diagonal(n, rho, rank), np.diag(h))
