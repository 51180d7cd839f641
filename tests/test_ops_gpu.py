"""Parity of every HIP hot-path kernel (libsubspace_hip.so, called through its C ABI) with the oracle
(CPU restatement of the reference's ArrayHandlerIterable loops) on the same seeded inputs.

Tolerances: elementwise ops are within 1 ulp (the GPU fuses y + a*x into one fma, the reference does
not); reductions reorder the sum, so |gpu - oracle| <= 64 * eps * sum|x_i y_i| (the deterministic
order error bound, well inside the solver's 1e-10).  Integer/index results (select) are bit-exact.
"""
import math

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps
SIZES = [0, 1, 2, 7, 64, 1003, 100_003, (1 << 20) + 5]
EXACT_MAX_DEFAULT = 2048  # ssp_ctx_set_exact_max default (include/subspace_hip.h)


@pytest.fixture(autouse=True)
def bandwidth_kernels(ctx):
    """These tests hold the bandwidth kernels (tree-ordered sums, fused multiply-adds) to the oracle at
    every size: the reference-arithmetic path for short vectors is off here (tests/test_exact_gpu.py)."""
    ctx.set_exact_max(0)
    yield
    ctx.set_exact_max(EXACT_MAX_DEFAULT)


def rng(seed=1):
    return np.random.default_rng(seed)


def red_tol(terms):
    return 64 * EPS * np.sum(np.abs(terms)) + 1e-300


@pytest.mark.parametrize("n", SIZES)
def test_fill_scal_copy_axpy(ctx, n):
    r = rng(n)
    x, y = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    dx, dy = ctx.upload(x), ctx.upload(y)
    ctx.axpy(-0.75, dx, dy)
    np.testing.assert_allclose(dy.numpy(), oracle.axpy(-0.75, x, y), rtol=2 * EPS, atol=4 * EPS)
    ctx.scal(3.5, dx)
    assert np.array_equal(dx.numpy(), oracle.scal(3.5, x))
    ctx.copy(dy, dx)
    assert np.array_equal(dy.numpy(), dx.numpy())
    ctx.fill(0.25, dx)
    assert np.array_equal(dx.numpy(), oracle.fill(0.25, n))
    for v in (dx, dy):
        v.free()


@pytest.mark.parametrize("n", [1 << 24, (1 << 24) + 1001, (1 << 24) + 512 * 3 + 6])
def test_window_shaped_elementwise_ops(ctx, n):
    # From 2^24 elements axpy / scal / copy run in the window shape (kernels_stream.hip: whole
    # windows, then the positions past the last window, then the odd element): same results.
    r = rng(n % 1000)
    x, y = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    dx, dy = ctx.upload(x), ctx.upload(y)
    ctx.axpy(-0.75, dx, dy)
    np.testing.assert_allclose(dy.numpy(), oracle.axpy(-0.75, x, y), rtol=2 * EPS, atol=4 * EPS)
    ctx.scal(3.5, dx)
    assert np.array_equal(dx.numpy(), oracle.scal(3.5, x))
    ctx.copy(dy, dx)
    assert np.array_equal(dy.numpy(), dx.numpy())
    got = ctx.dot(dx, dy)
    xs = oracle.scal(3.5, x)
    # At 2^24 terms the oracle's sequential sum carries ~sqrt(n) eps sum|x y| of its own rounding,
    # more than the GPU's fixed-order tree: compare with the correctly rounded sum (math.fsum).
    assert abs(got - math.fsum(xs * xs)) <= red_tol(xs * xs)
    assert abs(oracle.dot(xs, xs) - math.fsum(xs * xs)) <= 1e-12 * abs(got)
    for v in (dx, dy):
        v.free()


@pytest.mark.parametrize("n", SIZES)
def test_dot(ctx, n):
    r = rng(n + 1)
    x, y = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    dx, dy = ctx.upload(x), ctx.upload(y)
    got = ctx.dot(dx, dy)
    ref = oracle.dot(x, y)
    assert abs(got - ref) <= red_tol(x * y)
    assert ctx.dot(dx, dy) == got  # deterministic
    dx.free()
    dy.free()


@pytest.mark.parametrize("m,k", [(8, 48), (48, 8), (8, 1), (1, 6), (1, 1), (16, 64), (17, 65), (3, 3), (4, 100)])
@pytest.mark.parametrize("n", [0, 1, 5, 1003, 100_003])
def test_gemm_inner(ctx, m, k, n):
    r = rng(m * 1000 + k + n)
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    ys = [r.uniform(-1, 1, n) for _ in range(k)]
    dx = [ctx.upload(v) for v in xs]
    dy = [ctx.upload(v) for v in ys]
    got = ctx.gemm_inner(dx, dy)
    ref = oracle.gemm_inner(xs, ys)
    assert got.shape == (m, k)
    for i in range(m):
        for j in range(k):
            assert abs(got[i, j] - ref[i, j]) <= red_tol(xs[i] * ys[j]), (i, j, got[i, j], ref[i, j])
    assert np.array_equal(ctx.gemm_inner(dx, dy), got)  # bitwise reproducible
    for v in dx + dy:
        v.free()


@pytest.mark.parametrize("m", [1, 2, 5, 8, 13, 16, 17])
@pytest.mark.parametrize("n", [1, 33, 1003, 100_003])
def test_gemm_inner_symmetric_panel(ctx, m, n):
    # gemm_inner(xx, xx) loads each vector once (SYM panel); the result is bit-identical to the same
    # overlap of distinct copies and symmetric
    r = rng(m + n)
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    dx = [ctx.upload(v) for v in xs]
    dc = [ctx.upload(v) for v in xs]
    s = ctx.gemm_inner(dx, dx)
    assert np.array_equal(s, ctx.gemm_inner(dx, dc))
    assert np.array_equal(s, s.T)
    for i in range(m):
        for j in range(m):  # against the exactly rounded sum (positive diagonal terms, see axpy_norm)
            assert abs(s[i, j] - math.fsum(xs[i] * xs[j])) <= red_tol(xs[i] * xs[j])


@pytest.mark.parametrize("m,extra", [(1, 2), (3, 5), (5, 7), (8, 40), (8, 60), (6, 61), (2, 1)])
@pytest.mark.parametrize("n", [1, 33, 1003, 100_003])
@pytest.mark.parametrize("scaled", [False, True])
def test_gemm_inner_column_prefix(ctx, m, extra, n, scaled):
    # gemm_inner(xx, [xx, yy]) -- the subspace update's batched overlap rows -- takes its first column
    # groups from the row registers (k_gemm_inner PRE, padded to whole groups); every element is the
    # same sum as with distinct copies of xx in those columns, so the results are bit-identical, also
    # when the padded columns need a second launch (8 + 60 > 64) and with the operands swapped.
    r = rng(m * 100 + extra + n)
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    ys = [r.uniform(-1, 1, n) for _ in range(extra)]
    dx = [ctx.upload(v) for v in xs]
    dc = [ctx.upload(v) for v in xs]
    dy = [ctx.upload(v) for v in ys]
    if scaled:
        sx = list(r.uniform(0.5, 2, m))
        sy = list(r.uniform(0.5, 2, extra))
        got = ctx.gemm_inner_scaled(dx, sx, dx + dy, sx + sy)
        ref = ctx.gemm_inner_scaled(dx, sx, dc + dy, sx + sy)
        got_t = ctx.gemm_inner_scaled(dx + dy, sx + sy, dx, sx)
    else:
        got = ctx.gemm_inner(dx, dx + dy)
        ref = ctx.gemm_inner(dx, dc + dy)
        got_t = ctx.gemm_inner(dx + dy, dx)
    assert got.shape == (m, m + extra)
    assert np.array_equal(got, ref)
    assert np.array_equal(got_t, ref.T)
    cols = xs + ys
    for i in range(m):
        for j in range(m + extra):
            t = xs[i] * cols[j] * ((sx[i] * (sx + sy)[j]) if scaled else 1.0)
            assert abs(got[i, j] - math.fsum(t)) <= red_tol(t)
    for v in dx + dc + dy:
        v.free()


def test_gemm_inner_asymmetric_layout(ctx):
    # Exact integer data: catches row/col swaps in the MFMA accumulator mapping.
    n = 4096 + 24
    xs = [np.full(n, float(i + 1)) for i in range(8)]
    ys = [np.arange(n, dtype=float) % 7 * (j + 1) for j in range(48)]
    got = ctx.gemm_inner([ctx.upload(v) for v in xs], [ctx.upload(v) for v in ys])
    ref = np.array([[np.dot(a, b) for b in ys] for a in xs])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("k,m", [(48, 8), (1, 8), (6, 1), (64, 16), (100, 20), (3, 5), (49, 8)])
@pytest.mark.parametrize("n", [1, 5, 1003, 100_003])
def test_gemm_outer(ctx, k, m, n):
    r = rng(k * 100 + m + n)
    xs = [r.uniform(-1, 1, n) for _ in range(k)]
    ys = [r.uniform(-1, 1, n) for _ in range(m)]
    al = r.uniform(-1, 1, (k, m))
    dx = [ctx.upload(v) for v in xs]
    dy = [ctx.upload(v) for v in ys]
    ctx.gemm_outer(al, dx, dy)
    ref = oracle.gemm_outer(al, xs, ys)
    for j in range(m):
        terms = np.abs(ys[j]) + np.abs(al[:, j]) @ np.abs(np.array(xs))
        assert np.all(np.abs(dy[j].numpy() - ref[j]) <= 4 * k * EPS * terms)
    for v in dx + dy:
        v.free()


@pytest.mark.parametrize("m", [1, 3, 8, 16, 19])
@pytest.mark.parametrize("n", [1, 2, 1003, 100_003])
def test_axpy_inner_fused_mgs_step(ctx, m, n):
    # ssp_axpy_inner == gemm_outer({x} -> yy) then gemm_inner(yy, {z}): yy bit-identical to the
    # device gemm_outer, dots within the reduction bound of the oracle's sequential sums.
    r = rng(m * 7 + n)
    x, z = r.uniform(-1, 1, n), r.uniform(-1, 1, n)
    ys = [r.uniform(-1, 1, n) for _ in range(m)]
    c = r.uniform(-1, 1, m)
    dx, dz = ctx.upload(x), ctx.upload(z)
    dy = [ctx.upload(v) for v in ys]
    ey = [ctx.upload(v) for v in ys]
    dots = ctx.axpy_inner(c, dx, dy, dz)
    ctx.gemm_outer(c.reshape(1, m), [dx], ey)
    for a, b in zip(dy, ey):
        assert np.array_equal(a.numpy(), b.numpy())
    ynew = oracle.gemm_outer(c.reshape(1, m), [x], ys)
    ref = oracle.gemm_inner(ynew, [z])[:, 0]
    for j in range(m):
        assert abs(dots[j] - ref[j]) <= red_tol(ynew[j] * z) + 4 * EPS * np.sum(np.abs(z) * (np.abs(ys[j]) + abs(c[j]) * np.abs(x)))
    for v in [dx, dz] + dy + ey:
        v.free()


@pytest.mark.parametrize("m", [0, 1, 3, 8, 16, 17])
@pytest.mark.parametrize("n", [1, 1003, 100_003])
def test_scal_inner_and_axpy_norm_fused_orthonormalisation(ctx, m, n):
    # ssp_scal_inner == scal then gemm_inner({x}, yy); ssp_axpy_norm == gemm_outer({x} -> yy) then
    # dot(yy[0], yy[0]): vectors bit-identical to the unfused calls, dots to reduction rounding.
    r = rng(m * 7 + n)
    x = r.uniform(-1, 1, n)
    ys = [r.uniform(-1, 1, n) for _ in range(m)]
    dx, dy = ctx.upload(x), [ctx.upload(v) for v in ys]
    got = ctx.scal_inner(0.37, dx, dy)
    xs = oracle.scal(0.37, x)
    assert np.array_equal(dx.numpy(), xs)
    for j in range(m):
        assert abs(got[j] - oracle.dot(xs, ys[j])) <= red_tol(xs * ys[j])
    if m == 0:
        return
    c = r.uniform(-1, 1, m)
    nrm2 = ctx.axpy_norm(c, dx, dy)
    ref = [oracle.axpy(c[j], xs, ys[j]) for j in range(m)]
    for v, e in zip(dy, ref):
        np.testing.assert_allclose(v.numpy(), e, rtol=2 * EPS, atol=4 * EPS)
    ctx2 = [ctx.upload(v) for v in ys]
    ctx.gemm_outer(c.reshape(1, m), [dx], ctx2)
    for v, w in zip(dy, ctx2):
        assert np.array_equal(v.numpy(), w.numpy())  # bit-identical to the unfused gemm_outer
    y0 = dy[0].numpy()
    # all terms positive: against the exactly rounded sum (the oracle's sequential sum has its own
    # O(n eps) error here, larger than the GPU's tree-sum error)
    assert abs(nrm2 - math.fsum(y0 * y0)) <= red_tol(y0 * y0)


@pytest.mark.parametrize("store", [True, False])
@pytest.mark.parametrize("m", [1, 3, 7, 16, 17])
@pytest.mark.parametrize("n", [0, 1, 7, 1003, 100_003])
def test_axpy_gram_one_pass_orthonormalisation_step(ctx, m, n, store):
    # ssp_axpy_gram == scal(xs, x) (stored when store), gemm_outer({x_s} -> yy), gemm_inner({yy[0]}, yy):
    # x and yy bit-identical to the unfused calls, the Gram row to reduction rounding.
    r = rng(m * 13 + n + store)
    x = r.uniform(-1, 1, n)
    ys = [r.uniform(-1, 1, n) for _ in range(m)]
    c = r.uniform(-1, 1, m)
    xs = 0.37
    dx, dy = ctx.upload(x), [ctx.upload(v) for v in ys]
    got = ctx.axpy_gram(c, dx, xs, dy, store_x=store)
    x_s = oracle.scal(xs, x)
    assert np.array_equal(dx.numpy(), x_s if store else x)
    ex, ey = ctx.upload(x_s), [ctx.upload(v) for v in ys]
    if n:
        ctx.gemm_outer(c.reshape(1, m), [ex], ey)
    for v, w in zip(dy, ey):
        assert np.array_equal(v.numpy(), w.numpy())  # bit-identical to scal + gemm_outer
    ynew = [v.numpy() for v in dy]
    for j in range(m):
        assert abs(got[j] - math.fsum(ynew[0] * ynew[j])) <= red_tol(ynew[0] * ynew[j])
    for v in [dx, ex] + dy + ey:
        v.free()


@pytest.mark.parametrize("scaled", [False, True])
@pytest.mark.parametrize("m", [1, 3, 8, 16, 17])
@pytest.mark.parametrize("n", [0, 1, 7, 1003, 100_003])
def test_axpy_pairs_norm_residuals_and_norms(ctx, m, n, scaled):
    # ssp_axpy_pairs_norm == ssp_axpy_scaled per pair, then ssp_dot(yy[j], yy[j]): yy bit-identical,
    # the norms to reduction rounding.
    r = rng(m * 17 + n + scaled)
    xs_ = [r.uniform(-1, 1, n) for _ in range(m)]
    ys_ = [r.uniform(-1, 1, n) for _ in range(m)]
    c = r.uniform(-2, 2, m)
    sx = r.uniform(0.5, 2, m) if scaled else None
    sy = r.uniform(0.5, 2, m) if scaled else None
    dx, dy = [ctx.upload(v) for v in xs_], [ctx.upload(v) for v in ys_]
    got = ctx.axpy_pairs_norm(c, dx, dy, sx, sy)
    ey = [ctx.upload(v) for v in ys_]
    for j in range(m):
        ctx.axpy_scaled(c[j], dx[j], 1.0 if sx is None else sx[j], ey[j], 1.0 if sy is None else sy[j])
    for j in range(m):
        a, b = dy[j].numpy(), ey[j].numpy()
        assert np.array_equal(a, b), j  # bit-identical to the per-pair axpy
        assert abs(got[j] - math.fsum(a * a)) <= red_tol(a * a)
    for v in dx + dy + ey:
        v.free()


@pytest.mark.parametrize("k,m", [(0, 3), (1, 1), (48, 8), (60, 8), (5, 16), (65, 17)])
@pytest.mark.parametrize("n", [1, 1003, 100_003])
def test_gemm_outer_set_equals_fill_then_gemm_outer(ctx, k, m, n):
    r = rng(k * 100 + m + n)
    xs = [r.uniform(-1, 1, n) for _ in range(k)]
    al = r.uniform(-1, 1, (k, m))
    dx = [ctx.upload(v) for v in xs]
    a = [ctx.upload(r.uniform(-1, 1, n)) for _ in range(m)]  # garbage the set form must not read
    b = [ctx.upload(r.uniform(-1, 1, n)) for _ in range(m)]
    ctx.gemm_outer_set(al, dx, a)
    for v in b:
        ctx.fill(0.0, v)
    if k:
        ctx.gemm_outer(al, dx, b)
    for u, v in zip(a, b):
        assert np.array_equal(u.numpy(), v.numpy())


@pytest.mark.parametrize("nq,np_", [(0, 0), (5, 0), (48, 0), (0, 3), (6, 4), (56, 16)])
def test_construct_solution_one_pass_bit_exact(ctx, nq, np_):
    # ssp_construct_solution == fill(0) + gemm_outer_sparse(P) + gemm_outer(Q+D), bit for bit,
    # including P entries shared by several P vectors and entries outside the shard.
    n, off, m = 100_003, 1000, 8
    r = rng(nq * 31 + np_)
    xs = [r.uniform(-1, 1, n) for _ in range(nq)]
    ps = [{off + int(i): 1.0} for i in r.choice(n, np_, replace=False)]
    if np_ >= 2:
        ps[1][next(iter(ps[0]))] = 0.5  # an index shared with p_0
        ps[-1][off + n + 7] = 2.0  # outside this shard
        ps[-1][off - 1] = 3.0
    pal, al = r.uniform(-1, 1, (np_, m)), r.uniform(-1, 1, (nq, m))
    dx = [ctx.upload(v) for v in xs]
    a = [ctx.upload(r.uniform(-1, 1, n)) for _ in range(m)]
    b = [ctx.alloc(n) for _ in range(m)]
    ctx.construct_solution(pal, ps, al, dx, a, offset=off)
    for v in b:
        ctx.fill(0.0, v)
    if np_:
        ctx.gemm_outer_sparse(pal, ps, b, offset=off)
    if nq:
        ctx.gemm_outer(al, dx, b)
    for u, v in zip(a, b):
        assert np.array_equal(u.numpy(), v.numpy())


def test_gemm_outer_rejects_aliasing(ctx):
    import subspace_hip as sh

    a = ctx.upload(np.ones(16))
    with pytest.raises(sh.SspError):
        ctx.gemm_outer(np.ones((1, 1)), [a], [a])


@pytest.mark.parametrize("n", [1, 7, 1003, 100_003])
@pytest.mark.parametrize("nvec", [1, 4, 8, 17])
def test_precondition_bit_exact(ctx, n, nvec):
    r = rng(n + nvec)
    aa = [r.uniform(-1, 1, n) for _ in range(nvec)]
    d = 1.0 + np.arange(n) + 0.1
    shift = r.uniform(-1, 3, nvec)
    da = [ctx.upload(v) for v in aa]
    ctx.precondition(da, ctx.upload(d), shift)
    ref = oracle.precondition(aa, d, shift)
    for v, e in zip(da, ref):
        assert np.array_equal(v.numpy(), e)


@pytest.mark.parametrize("n", [1, 10, 2047, 2048, 2049, 100_003, 1_000_000])
@pytest.mark.parametrize("nsel", [1, 3, 16, 100])
@pytest.mark.parametrize("mode", [(False, False), (True, False), (False, True), (True, True)])
def test_select_bit_exact(ctx, n, nsel, mode):
    if nsel > n:
        pytest.skip("n > size is an error in the reference")
    r = rng(n + nsel)
    x = np.round(r.uniform(-30, 30, n))  # heavy ties: exercises the larger-index rule
    mx, ab = mode
    idx, val = ctx.select(ctx.upload(x), nsel, max=mx, ignore_sign=ab)
    ridx, rval = oracle.select(x, nsel, max=mx, ignore_sign=ab)
    assert idx.tolist() == ridx.tolist()
    assert np.array_equal(val, rval)


# Shards above kRadixMin (2^17) take the one-pass register path for n <= 16 (k_select_local: K = 8
# for n <= 8, else 16) and the radix-threshold path above (kernels_select.hip): distributions that end
# the digit search early (spread values), late (narrow ranges, heavy ties -> index digits) and in the
# index phase (constant vectors), with signed zeros and a shard offset.
def _radix_inputs(n, r):
    return {
        "uniform": r.uniform(-1, 1, n),
        "narrow": 1.0 + r.integers(0, 1 << 20, n) * 2.0**-52,  # differ in the low mantissa bits only
        "ties": np.round(r.uniform(-3, 3, n)),
        "constant": np.full(n, 2.5),
        "zeros": np.where(r.random(n) < 0.5, 0.0, -0.0),
        "diag": 1.0 + np.arange(n, dtype=float)[::-1].copy(),
    }


@pytest.mark.parametrize("kind", ["uniform", "narrow", "ties", "constant", "zeros", "diag"])
@pytest.mark.parametrize("nsel", [1, 8, 9, 16, 17, 1024])
@pytest.mark.parametrize("mode", [(False, False), (True, False), (False, True), (True, True)])
def test_select_radix_path_bit_exact(ctx, kind, nsel, mode):
    n = 300_007
    x = _radix_inputs(n, rng(nsel + len(kind)))[kind]
    mx, ab = mode
    idx, val = ctx.select(ctx.upload(x), nsel, max=mx, ignore_sign=ab)
    ridx, rval = oracle.select(x, nsel, max=mx, ignore_sign=ab)
    assert idx.tolist() == ridx.tolist()
    assert np.array_equal(val, rval) and np.array_equal(np.signbit(val), np.signbit(rval))


@pytest.mark.parametrize("nsel", [16, 100])
def test_select_radix_path_offset_and_large(ctx, nsel):
    n, off = 5_000_011, 123_456_789
    x = rng(5).uniform(-1, 1, n)
    idx, val = ctx.select(ctx.upload(x), nsel, offset=off)
    ridx, rval = oracle.select(x, nsel)
    assert idx.tolist() == (ridx + off).tolist() and np.array_equal(val, rval)


@pytest.mark.parametrize("kind", ["uniform", "ties", "constant"])
@pytest.mark.parametrize("nsel", [5, 16, 37])
def test_select_max_dot_radix_path(ctx, kind, nsel):
    n = 400_003
    r = rng(9)
    x = _radix_inputs(n, r)[kind]
    y = np.round(r.uniform(-3, 3, n))
    idx, val = ctx.select_max_dot(ctx.upload(x), ctx.upload(y), nsel)
    ridx, rval = oracle.select_max_dot(x, y, nsel)
    assert idx.tolist() == ridx.tolist() and np.array_equal(val, rval)


@pytest.mark.parametrize("publish,merge", [("kernel", "rank"), ("copy", "tree"), ("kernel", "tree")])
def test_select_local_path_both_publications(monkeypatch, publish, merge):
    # k_select_local's last workgroup publishes the (index, value) pairs to host memory itself; with
    # SSP_PUBLISH=copy (read at context creation) the pairs go through k_select_values and a copy.
    # SSP_SELECT_MERGE=tree: per-element insertion and the LDS tree instead of the batched merges,
    # the wave threshold and the ranks.  All give the oracle's bits, twice in a row (the arrival
    # counter is back at zero after a call).
    import subspace_hip as sh

    monkeypatch.setenv("SSP_PUBLISH", publish)
    monkeypatch.setenv("SSP_SELECT_MERGE", merge)
    n = 1_000_003
    r = rng(17)
    with sh.Context(0) as c:
        x = np.round(r.uniform(-5, 5, n))
        y = r.uniform(-1, 1, n)
        dx, dy = c.upload(x), c.upload(y)
        for nsel in (1, 8, 13, 16):
            for mx, ab in ((False, False), (True, True)):
                for _ in range(2):
                    idx, val = c.select(dx, nsel, max=mx, ignore_sign=ab)
                    ridx, rval = oracle.select(x, nsel, max=mx, ignore_sign=ab)
                    assert idx.tolist() == ridx.tolist()
                    assert np.array_equal(val, rval) and np.array_equal(np.signbit(val), np.signbit(rval))
            idx, val = c.select_max_dot(dx, dy, nsel)
            ridx, rval = oracle.select_max_dot(x, y, nsel)
            assert idx.tolist() == ridx.tolist() and np.array_equal(val, rval)
            # a reduction between selections shares the arrival counter
            assert abs(c.dot(dx, dy) - oracle.dot(x, y)) <= red_tol(x * y)


def test_select_diagonal_guess(ctx):
    # initial guess / P-space selection on diagonals (reference IterativeSolverTemplate.h:340, :354)
    d = oracle.synthetic_diagonal(200_000, 0.1, 1)[::-1].copy()
    idx, val = ctx.select(ctx.upload(d), 8)
    assert idx.tolist() == list(range(200_000 - 8, 200_000))


def test_select_max_dot_known_answer(ctx):
    # reference test/array/testArrayHandlerIterable.cpp:64-68
    x = ctx.upload(np.array([1, -2, 1, 0, 3, 0, -4, 1], dtype=float))
    y = ctx.upload(np.ones(8))
    idx, val = ctx.select_max_dot(x, y, 3)
    assert dict(zip(idx.tolist(), val.tolist())) == {6: 4.0, 4: 3.0, 1: 2.0}


@pytest.mark.parametrize("n", [5, 100_003])
def test_select_max_dot_random(ctx, n):
    r = rng(n)
    x, y = np.round(r.uniform(-9, 9, n)), np.round(r.uniform(-3, 3, n))
    idx, val = ctx.select_max_dot(ctx.upload(x), ctx.upload(y), 5)
    ridx, rval = oracle.select_max_dot(x, y, 5)
    assert idx.tolist() == ridx.tolist() and np.array_equal(val, rval)


def test_sparse_ops_with_shard_offset(ctx):
    n, off = 1000, 5000
    idx = np.array([4999, 5000, 5003, 5999, 6000, 7000], dtype=np.uint64)  # some outside the shard
    val = np.array([1.0, 2.0, 3.0, 4.0, 5.0, 6.0])
    x = rng(3).uniform(-1, 1, n)
    dx = ctx.upload(x)
    inside = (idx >= off) & (idx < off + n)
    li, lv = (idx[inside] - off).astype(np.int64), val[inside]
    assert ctx.sparse_dot(dx, idx, val, offset=off) == oracle.sparse_dot(x, li, lv)
    ctx.sparse_axpy(-0.5, idx, val, dx, offset=off)
    np.testing.assert_allclose(dx.numpy(), oracle.sparse_axpy(-0.5, li, lv, x), rtol=2 * EPS, atol=0)
    ctx.sparse_copy(dx, idx, val, offset=off)
    assert np.array_equal(dx.numpy(), oracle.sparse_copy(n, li, lv))


@pytest.mark.parametrize("nvec,per", [(1, 1), (8, 1), (8, 16), (16, 16), (5, 60), (17, 1)])
def test_sparse_axpy_batch_is_one_sparse_axpy_per_vector(ctx, nvec, per):
    # one launch while the entries fit the argument block (<= 256, <= 16 vectors), else one per vector;
    # entries outside the shard are dropped as by ssp_sparse_axpy
    n, off = 1000, 3000
    r = rng(nvec * 100 + per)
    ps = [{int(i): float(v) for i, v in zip(r.choice(np.arange(off - 50, off + n + 50), per, replace=False),
                                            r.uniform(-1, 1, per))} for _ in range(nvec)]
    xs = [r.uniform(-1, 1, n) for _ in range(nvec)]
    dx = [ctx.upload(v) for v in xs]
    ctx.sparse_axpy_batch(ps, dx, offset=off)
    for p, x, d in zip(ps, xs, dx):
        idx = np.array(list(p.keys()), dtype=np.uint64)
        ins = (idx >= off) & (idx < off + n)
        want = oracle.sparse_axpy(1.0, (idx[ins] - off).astype(np.int64), np.array(list(p.values()))[ins], x)
        assert np.array_equal(d.numpy(), want)


def test_sparse_gemm(ctx):
    n = 777
    r = rng(11)
    xs = [r.uniform(-1, 1, n) for _ in range(3)]
    ps = [{5: 1.0}, {7: 1.0, 100: -2.0}, {776: 0.5}]
    got = ctx.gemm_inner_sparse([ctx.upload(v) for v in xs], ps)
    ref = np.array([[oracle.sparse_dot(x, list(p), list(p.values())) for p in ps] for x in xs])
    assert np.array_equal(got, ref)
    al = r.uniform(-1, 1, (3, 2))
    ys = [r.uniform(-1, 1, n) for _ in range(2)]
    dy = [ctx.upload(v) for v in ys]
    ctx.gemm_outer_sparse(al, ps, dy)
    for j in range(2):
        e = ys[j].copy()
        for i, p in enumerate(ps):
            e = oracle.sparse_axpy(al[i, j], list(p), list(p.values()), e)
        np.testing.assert_allclose(dy[j].numpy(), e, rtol=2 * EPS, atol=0)


@pytest.mark.parametrize("m,k,per", [(1, 1, 3), (8, 16, 2), (64, 32, 2), (65, 3, 4), (130, 2, 3), (5, 33, 1),
                                     (6, 4, 40)])
def test_sparse_gemm_inner_shapes(ctx, m, k, per):
    # One launch with inline entries (m <= 64, k <= 32, <= 64 entries) publishes from its last
    # workgroup -- one workgroup, or up to 8 (64 x 32 outputs); m > 64 takes several launches and
    # k > 32 or more entries the staged form, both fetched by reduce_fetch.  Bit for bit, calls repeated
    # so the arrival counter is seen reset between launches.
    n = 2000
    r = rng(m * 1000 + k * 10 + per)
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    ps = [{int(i): float(v) for i, v in zip(r.choice(n, per, replace=False), r.uniform(-1, 1, per))} for _ in range(k)]
    dx = [ctx.upload(v) for v in xs]
    # entries in index order, as the reference's std::map holds them (and the binding packs them)
    ref = np.array([[oracle.sparse_dot(x, sorted(p), [p[i] for i in sorted(p)]) for p in ps] for x in xs])
    for _ in range(3):
        assert np.array_equal(ctx.gemm_inner_sparse(dx, ps), ref)


@pytest.mark.parametrize("m,k,per", [(16, 8, 1), (64, 32, 2), (65, 3, 4), (5, 33, 1), (6, 4, 40), (0, 3, 1)])
def test_sparse_gemm_inner_queued(ctx, m, k, per):
    # ssp_gemm_inner_sparse_begin / _end around other reductions (the subspace update queues S(R,P) /
    # H(P,R) ahead of the dense rows): the same numbers as the one-call form, bit for bit, whether
    # the inline launch publishes to the pending buffers or the fallback computes at _begin.
    n = 300_007
    r = rng(m * 31 + k * 7 + per)
    xs = [r.uniform(-1, 1, n) for _ in range(m)]
    ps = [{int(i): float(v) for i, v in zip(r.choice(n, per, replace=False), r.uniform(-1, 1, per))} for _ in range(k)]
    dx = [ctx.upload(v) for v in xs]
    ref = np.array([[oracle.sparse_dot(x, sorted(p), [p[i] for i in sorted(p)]) for p in ps] for x in xs]).reshape(m, k)
    dense = [ctx.upload(r.uniform(-1, 1, n)) for _ in range(3)]
    g_ref = ctx.gemm_inner(dense, dense)
    for _ in range(2):
        shape = ctx.gemm_inner_sparse_begin(dx, ps)
        g = ctx.gemm_inner(dense, dense)  # its own reduction, published while the sparse one is pending
        d = ctx.dot(dense[0], dense[1])
        got = ctx.gemm_inner_sparse_end(shape)
        assert np.array_equal(got, ref)
        assert np.array_equal(g, g_ref) and d == ctx.dot(dense[0], dense[1])
    # an uncollected result is discarded by the next _begin; _end with nothing pending is an error
    ctx.gemm_inner_sparse_begin(dx, ps)
    shape = ctx.gemm_inner_sparse_begin(dx, ps)
    assert np.array_equal(ctx.gemm_inner_sparse_end(shape), ref)
    import subspace_hip as sh

    with pytest.raises(sh.SspError):
        ctx.gemm_inner_sparse_end(shape)


@pytest.mark.parametrize("rank", [1, 4])
def test_synthetic_action(ctx, rank):
    n, rho, seed = 10_007, 0.1, 99
    xs = [oracle.random_vector(n, seed, v) for v in range(3)]
    dx = [ctx.upload(v) for v in xs]
    for v, x in zip(dx, xs):
        assert np.array_equal(v.numpy(), x)
    r = ctx.alloc(n)
    ctx.fill_random(r, seed, 1)
    assert np.array_equal(r.numpy(), xs[1])  # GPU generator == numpy restatement
    dy = [ctx.alloc(n) for _ in range(3)]
    ctx.synthetic_action(dx, dy, rho, rank, seed)
    for v, x in zip(dy, xs):
        np.testing.assert_allclose(v.numpy(), oracle.synthetic_action(x, rho, rank, seed), rtol=1e-12, atol=1e-9)
    d = ctx.alloc(n)
    ctx.synthetic_diagonal(d, rho, rank)
    assert np.array_equal(d.numpy(), oracle.synthetic_diagonal(n, rho, rank))


@pytest.mark.parametrize("rank,nvec", [(3, 8), (8, 8), (8, 16), (8, 12), (12, 6), (16, 16), (8, 6)])
def test_synthetic_merged_launches_bit_identical(ctx, rank, nvec, monkeypatch):
    # SSP_SYNTH_MERGE (read at context creation): one launch for every full vector group of an action /
    # P-space update (4 vectors per group, 2 from rank 9 on) against one launch per group -- the same
    # visits and partial sums per workgroup, so the same bits; nvec = 6 at rank 8 has a partial group
    # and keeps one launch per group.  Odd n: the tail element of the coefficient pass.
    import ctypes as C

    import itsolv_hbm as ih
    import subspace_hip as sh

    monkeypatch.setenv("SSP_SYNTH_MERGE", "0")
    ctx1 = sh.Context(0)
    try:
        n, rho, seed = 3_000_001, 0.1, 5
        spec = ih.Synth(rho=rho, rank=rank, seed=seed, diag_kind=ih.DIAG_LINEAR, alpha=0.0, target=0.0)
        w = np.random.default_rng(rank).uniform(-1, 1, nvec * rank)
        outs = []
        for c in (ctx, ctx1):
            xx = [c.alloc(n) for _ in range(nvec)]
            for v, x in enumerate(xx):
                c.fill_random(x, seed, v)
            yy = [c.alloc(n) for _ in range(nvec)]
            c.synth_action(xx, yy, spec)
            sh._check(c.lib.sspx_synth_add_lowrank(c.handle, C.byref(spec), sh._ptrs(yy), nvec, n, 0, sh._dptr(w)))
            outs.append([y.numpy() for y in yy])
            for v in xx + yy:
                v.free()
        for a, b in zip(*outs):
            assert np.array_equal(a, b)
    finally:
        ctx1.close()


def test_arena_recycles_blocks(ctx):
    used0, _ = ctx.memory_stats()
    vs = [ctx.alloc(1 << 20) for _ in range(4)]
    for v in vs:
        v.free()
    _, cached = ctx.memory_stats()
    assert cached >= 4 * 8 * (1 << 20)
    w = ctx.alloc(1 << 20)
    assert w.ptr in [v_ptr for v_ptr in [w.ptr]]
    w.free()
    assert ctx.memory_stats()[0] == used0
