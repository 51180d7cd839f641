"""The reference's own arithmetic on short vectors (ssp_ctx_set_exact_max, kernels_exact.hip; 2048 local
elements by default, raised to 16384 here): every dot a sequential sum in index order and every y = alpha x + y
rounded twice, so each entry point is the oracle's restated loop (ArrayHandlerIterable.h:65-82,
util/gemm.h:257-279) BIT FOR BIT, and a whole solve on the reference's own test problems -- with the
reference's sequential MGS, which the HBM handlers keep below fused_min_size() -- is the reference
CPU path step for step, to the last bit of every eigenvalue, residual norm and solution.

Bar: np.array_equal on the raw values (no tolerance).
"""
import numpy as np
import pytest

import itsolv_hbm as ih
import oracle

pytestmark = pytest.mark.gpu
SIZES = [1, 2, 7, 64, 1003, 4097, 16384]


def bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def same(a, b):
    return np.array_equal(bits(a), bits(b))


@pytest.fixture
def exact(ctx):
    ctx.set_exact_max(16384)
    yield ctx
    ctx.set_exact_max(2048)  # the default (include/subspace_hip.h)


@pytest.mark.parametrize("n", SIZES)
def test_elementwise_and_dots_are_the_reference_loops(exact, n):
    ctx = exact
    r = np.random.default_rng(n)
    x, y = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    dx, dy = ctx.upload(x), ctx.upload(y)
    assert same(ctx.dot(dx, dy), oracle.dot(x, y))
    assert same(ctx.dot(dx, dx), oracle.dot(x, x))
    ctx.axpy(-0.75, dx, dy)
    assert same(dy.numpy(), oracle.axpy(-0.75, x, y))
    # deferred scales: the kernel sees the values an eager scal would have stored
    y2 = oracle.axpy(-0.75, x, y)
    ctx.axpy_scaled(0.3, dx, 1.7, dy, -0.9)
    assert same(dy.numpy(), oracle.axpy(0.3, oracle.scal(1.7, x), oracle.scal(-0.9, y2)))
    assert same(ctx.dot_scaled(dx, 1.7, dy, 0.5), oracle.dot(oracle.scal(1.7, x), oracle.scal(0.5, dy.numpy())))
    for v in (dx, dy):
        v.free()


@pytest.mark.parametrize("m,k", [(1, 1), (1, 2), (3, 5), (8, 48), (17, 3)])
@pytest.mark.parametrize("n", [1, 1003, 16384])
def test_gemm_inner_and_outer_are_the_reference_loops(exact, m, k, n):
    ctx = exact
    r = np.random.default_rng(m * 100 + k + n)
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    ys = [r.uniform(-1, 1, n) for _ in range(k)]
    dx, dy = [ctx.upload(v) for v in xs], [ctx.upload(v) for v in ys]
    assert same(ctx.gemm_inner(dx, dy), oracle.gemm_inner(xs, ys))
    assert same(ctx.gemm_inner(dx, dx), oracle.gemm_inner(xs, xs))
    sx = r.uniform(0.5, 2, m)
    assert same(ctx.gemm_inner_scaled(dx, sx, dy, None), oracle.gemm_inner([oracle.scal(s, v) for s, v in zip(sx, xs)], ys))
    al = r.uniform(-1, 1, (m, k))
    ctx.gemm_outer(al, dx, dy)
    want = oracle.gemm_outer(al, xs, ys)
    for v, w in zip(dy, want):
        assert same(v.numpy(), w)
    ctx.gemm_outer_set(al, dx, dy)
    want = oracle.gemm_outer(al, xs, [np.zeros(n)] * k)
    for v, w in zip(dy, want):
        assert same(v.numpy(), w)
    for v in dx + dy:
        v.free()


@pytest.mark.parametrize("m", [1, 3, 16, 17])
@pytest.mark.parametrize("n", [1, 7, 1003, 16384])
def test_fused_entry_points_are_their_reference_sequences(exact, m, n):
    ctx = exact
    r = np.random.default_rng(m * 7 + n)
    x, z = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    ys = [r.uniform(-1, 1, n) for _ in range(m)]
    c = r.uniform(-1, 1, m)
    # axpy_inner: gemm_outer({x} -> yy), then <yy_j, z>
    dx, dz, dy = ctx.upload(x), ctx.upload(z), [ctx.upload(v) for v in ys]
    got = ctx.axpy_inner(c, dx, dy, dz)
    ynew = oracle.gemm_outer(c.reshape(1, m), [x], ys)
    assert same(got, oracle.gemm_inner(ynew, [z])[:, 0])
    for v, w in zip(dy, ynew):
        assert same(v.numpy(), w)
    # scal_inner: scal(x), then <x, yy_j>;  axpy_norm: gemm_outer, then <yy_0, yy_0>
    got = ctx.scal_inner(0.37, dx, dy)
    xs = oracle.scal(0.37, x)
    assert same(dx.numpy(), xs) and same(got, oracle.gemm_inner([xs], ynew)[0])
    nrm = ctx.axpy_norm(c, dx, dy)
    y2 = oracle.gemm_outer(c.reshape(1, m), [xs], ynew)
    assert same(nrm, oracle.dot(y2[0], y2[0]))
    # axpy_gram: x_s = 0.6 x (stored), gemm_outer({x_s} -> yy), then <yy_0, yy_j>
    got = ctx.axpy_gram(c, dx, 0.6, dy, store_x=True)
    x3 = oracle.scal(0.6, xs)
    y3 = oracle.gemm_outer(c.reshape(1, m), [x3], y2)
    assert same(dx.numpy(), x3) and same(got, oracle.gemm_inner([y3[0]], y3)[0])
    # axpy_pairs_norm: y_j = ys_j y_j + c_j (xs_j x_j) per pair, then <y_j, y_j>
    xx = [r.uniform(-1, 1, n) for _ in range(m)]
    dxx = [ctx.upload(v) for v in xx]
    sx, sy = r.uniform(0.5, 2, m), r.uniform(0.5, 2, m)
    got = ctx.axpy_pairs_norm(c, dxx, dy, sx, sy)
    y4 = [oracle.axpy(c[j], oracle.scal(sx[j], xx[j]), oracle.scal(sy[j], y3[j])) for j in range(m)]
    for j in range(m):
        assert same(dy[j].numpy(), y4[j]), j
        assert same(got[j], oracle.dot(y4[j], y4[j])), j
    for v in [dx, dz] + dy + dxx:
        v.free()


@pytest.mark.parametrize("n", [7, 1003])
def test_construct_solution_with_p_space_is_the_reference_sequence(exact, n):
    # fill(0), the sparse gemm_outer over P (entries in order), then the dense gemm_outer: bit for bit
    ctx = exact
    r = np.random.default_rng(n)
    k, m = 4, 3
    xs = [r.uniform(-1, 1, n) for _ in range(k)]
    ps = [{1: 0.5, n - 1: -1.25}, {3 % n: 2.0}, {1: 0.75}]
    pa, al = r.uniform(-1, 1, (len(ps), m)), r.uniform(-1, 1, (k, m))
    dx, dy = [ctx.upload(v) for v in xs], [ctx.alloc(n) for _ in range(m)]
    ctx.construct_solution(pa, ps, al, dx, dy)
    want = [np.zeros(n) for _ in range(m)]
    for i, p in enumerate(ps):
        idx, val = np.array(list(p.keys()), dtype=np.uint64), np.array(list(p.values()))
        for j in range(m):
            want[j] = oracle.sparse_axpy(pa[i, j], idx, val, want[j])
    want = oracle.gemm_outer(al, xs, want)
    for v, w in zip(dy, want):
        assert same(v.numpy(), w)


def test_exact_max_zero_selects_the_bandwidth_kernels(exact):
    # Above the limit (or with 0) the parallel kernels run: equal within the reduction bound, and the
    # limit is per context and per call.
    ctx = exact
    n = 1003
    r = np.random.default_rng(5)
    x, y = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    dx, dy = ctx.upload(x), ctx.upload(y)
    seq = ctx.dot(dx, dy)
    ctx.set_exact_max(0)
    par = ctx.dot(dx, dy)
    assert abs(par - seq) <= 64 * np.finfo(float).eps * np.sum(np.abs(x * y))
    ctx.set_exact_max(n)
    assert same(ctx.dot(dx, dy), seq)
    ctx.set_exact_max(n - 1)
    assert same(ctx.dot(dx, dy), par)


# ---- whole solves: the reference CPU path, bit for bit ---------------------------------------------
def hamiltonian(name, split):
    from test_solver_gpu import hamiltonian as h

    return h(name, split)


def same_solve(g, c, fields=("eigenvalues", "errors")):
    assert g["converged"] == c["converged"]
    assert g["iterations"] == c["iterations"], (g["iterations"], c["iterations"])
    for f in ("r_creations", "q_creations", "redundant_params", "null_params"):
        if f in c:
            assert g[f] == c[f], f
    for f in fields:
        if f in c:
            assert same(g[f], c[f]), (f, g[f], c[f])
    tg, tc = g.get("trace"), c.get("trace")
    if tg and tc:
        for key in tc:
            if key in tg:
                assert np.array_equal(np.asarray(tg[key]), np.asarray(tc[key])), key


@pytest.mark.parametrize("name,split", [("he", 0.0), ("hf", 1e-8), ("bh", 1e-8)])
@pytest.mark.parametrize("nroot,np_", [(1, 0), (3, 0), (3, 6)])
def test_fixture_davidson_is_the_reference_path(exact, name, split, nroot, np_):
    if name == "he" and nroot > 1:
        pytest.skip("degenerate pair in he")
    h = hamiltonian(name, split)
    kw = dict(nroots=nroot, max_p=np_, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
    g, c = ih.davidson_dense(exact, h, **kw), oracle.davidson_dense(h, **kw)
    same_solve(g, c, ("eigenvalues", "errors", "solutions"))


@pytest.mark.parametrize("n,rank,rho,seed", [(1000, 1, 0.1, 3), (1000, 3, 0.01, 3), (3000, 3, 0.01, 3)])
def test_diis_is_the_reference_path(exact, n, rank, rho, seed):
    # (1000, 1, 0.1) is the case whose step count the reference itself changes from 13 to 68 when only
    # its summation order changes (test_solver_gpu.py): with the reference's arithmetic the GPU takes
    # its 13 steps to the last bit.
    kw = dict(convergence_threshold=1e-8, max_size_qspace=6)
    g, c = ih.diis_synthetic(exact, n, rho, rank, seed, **kw), oracle.diis_synthetic(n, rho, rank, seed, **kw)
    same_solve(g, c, ("errors", "x"))


@pytest.mark.parametrize("nroot,np_", [(1, 0), (4, 0), (4, 8)])
def test_synthetic_davidson_short_vectors_is_the_reference_path(exact, nroot, np_):
    n, rho, rank, seed = 10_007, 0.1, 4, 20251015
    kw = dict(nroots=nroot, max_p=np_, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
    g = ih.davidson_synthetic(exact, n, rho, rank, seed, **kw)
    c = oracle.davidson_synthetic(n, rho, rank, seed, **kw)
    same_solve(g, c, ("eigenvalues", "errors", "residual_norms"))


@pytest.mark.parametrize("n,nroot", [(12, 3), (33, 13)])
def test_linear_equations_is_the_reference_path(exact, n, nroot):
    from test_solver_oracle import simple_system

    a, rhs = simple_system(n, nroot)
    kw = dict(nroots=nroot, convergence_threshold=1e-10)
    g, c = ih.linear_equations_dense(exact, a, rhs, **kw), oracle.linear_equations_dense(a, rhs, **kw)
    same_solve(g, c, ("errors", "x"))


@pytest.mark.parametrize("n,alg", [(4, "BFGS"), (100, "BFGS"), (20, "SD")])
def test_optimize_is_the_reference_path(exact, n, alg):
    from test_solver_oracle import rayleigh_matrix

    m = rayleigh_matrix(n, 0.01)
    kw = dict(convergence_threshold=1e-6 if n > 4 else 1e-8, max_iter=200)
    g, c = ih.optimize_dense(exact, m, alg, **kw), oracle.optimize_dense(m, alg, **kw)
    same_solve(g, c, ("eigenvalues", "x"))


@pytest.mark.parametrize("name", ["C1_rank1", "C1_rank8"])
def test_c1_traces_are_the_committed_reference_trace(exact, name):
    # BASELINE config C1 (N = 1e4): the committed per-iteration trace of the reference CPU path
    # (tests/golden/traces.json, JSON floats round-trip exactly), every value to the last bit.
    from trace_check import T

    ref = T[name]
    c = ref["case"]
    g = ih.davidson_synthetic(exact, c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **ref["options"])
    assert g["iterations"] == ref["iterations"] and g["converged"] == ref["converged"]
    assert g["r_creations"] == ref["r_creations"] and g["q_creations"] == ref["q_creations"]
    assert same(g["eigenvalues"], ref["eigenvalues"]) and same(g["errors"], ref["errors"])
    for key in ("eigenvalues", "errors", "nq", "nwork"):
        assert np.array_equal(np.asarray(g["trace"][key]), np.asarray(ref["trace"][key])), key


@pytest.mark.parametrize("n", [7, 1003])
def test_block_update_is_the_reference_sequence(exact, n):
    # yy[j] = ys[j] yy[j] (the eager scal), then the sparse gemm_outer over P, then the dense gemm_outer
    # over the scaled sources: bit for bit (the block Gram-Schmidt update's arithmetic on short vectors)
    ctx = exact
    r = np.random.default_rng(n + 1)
    k, m = 3, 4
    xs = [r.uniform(-1, 1, n) for _ in range(k)]
    ys = [r.uniform(-1, 1, n) for _ in range(m)]
    ps = [{0: 1.0}, {n - 1: -0.5, 2 % n: 0.25}]
    pa, al = r.uniform(-1, 1, (len(ps), m)), r.uniform(-1, 1, (k, m))
    sx, sy = r.uniform(0.5, 2, k), r.uniform(0.5, 2, m)
    dx, dy = [ctx.upload(v) for v in xs], [ctx.upload(v) for v in ys]
    ctx.block_update(pa, ps, al, dx, sx, dy, sy)
    want = [oracle.scal(sy[j], ys[j]) for j in range(m)]
    for i, p in enumerate(ps):
        idx, val = np.array(list(p.keys()), dtype=np.uint64), np.array(list(p.values()))
        for j in range(m):
            want[j] = oracle.sparse_axpy(pa[i, j], idx, val, want[j])
    want = oracle.gemm_outer(al, [oracle.scal(s, v) for s, v in zip(sx, xs)], want)
    for v, w in zip(dy, want):
        assert same(v.numpy(), w)
