"""Deferred scal on the MI355X (include/subspace_hip.h *_scaled, itsolv_hbm/hbm_vec.h Vec::scale_by).

The handlers' scal (reference ArrayHandlerIterable.h:54-57) is not a pass over the vector: the next
kernel that reads the vector multiplies each element by the pending scale as it loads it.  x * s is
the one rounding the eager scal stores, so every scaled entry point must equal -- bit for bit,
signed zeros included -- ssp_scal(s) on each operand followed by the unscaled call.  Covered: every
kernel shape the entry points launch (stride and window element-wise shapes, the MFMA panel, the
symmetric panel, the VALU row kernel, gemm_outer with argument-block and device alphas and more
than 64 sources, the sparse panels, construct_solution and the block update with P indices,
the synthetic action) at odd lengths.
"""
import numpy as np
import pytest

import itsolv_hbm as ih
import subspace_hip as sh

pytestmark = pytest.mark.gpu
EXACT_MAX_DEFAULT = 2048  # ssp_ctx_set_exact_max default (include/subspace_hip.h)


@pytest.fixture(autouse=True)
def bandwidth_kernels(ctx):
    """These tests hold the bandwidth kernels (tree-ordered sums, fused multiply-adds) to the oracle at
    every size: the reference-arithmetic path for short vectors is off here (tests/test_exact_gpu.py)."""
    ctx.set_exact_max(0)
    yield
    ctx.set_exact_max(EXACT_MAX_DEFAULT)


N_SMALL = 100_003
N_WIN = (1 << 24) + 5  # the window shape of the element-wise kernels


def bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def rand(rng, n, zeros=True):
    v = rng.uniform(-1, 1, n)
    if zeros:
        v[::997] = 0.0  # x * negative scale = -0
    return v


def scaled_copies(ctx, vals, scales):
    """(raw device vectors, eagerly scaled device vectors)."""
    raw = [ctx.upload(v) for v in vals]
    eag = [ctx.upload(v) for v in vals]
    for e, s in zip(eag, scales):
        if s != 1.0:
            ctx.scal(s, e)
    return raw, eag


@pytest.mark.parametrize("n", [N_SMALL, N_WIN])
def test_scal_copy_axpy_dot(ctx, n):
    rng = np.random.default_rng(1)
    x, y = rand(rng, n), rand(rng, n)
    for xs, ys in [(-0.37, 1.0), (1.0, 2.5), (-0.37, 2.5), (1.0, 1.0)]:
        (rx, ry), (ex, ey) = scaled_copies(ctx, [x, y], [xs, ys])
        out = ctx.alloc(n)
        ctx.scal_copy(xs, out, rx)
        assert np.array_equal(bits(out.numpy()), bits(ex.numpy())), "scal_copy"
        assert ctx.dot_scaled(rx, xs, ry, ys) == ctx.dot(ex, ey), "dot"
        assert ctx.dot_scaled(rx, xs, rx, xs) == ctx.dot(ex, ex), "norm"
        ctx.axpy_scaled(0.75, rx, xs, ry, ys)
        ctx.axpy(0.75, ex, ey)
        assert np.array_equal(bits(ry.numpy()), bits(ey.numpy())), "axpy"


@pytest.mark.parametrize("m,k", [(8, 48), (16, 64), (1, 1), (1, 2), (2, 1), (3, 70), (12, 5)])
def test_gemm_inner_scaled(ctx, m, k):
    rng = np.random.default_rng(m * 100 + k)
    xv = [rand(rng, N_SMALL) for _ in range(m)]
    yv = [rand(rng, N_SMALL) for _ in range(k)]
    xs = rng.choice([1.0, -0.5, 3.25, 0.1], m)
    ys = rng.choice([1.0, -0.5, 3.25, 0.1], k)
    rx, ex = scaled_copies(ctx, xv, xs)
    ry, ey = scaled_copies(ctx, yv, ys)
    got = ctx.gemm_inner_scaled(rx, xs, ry, ys)
    want = ctx.gemm_inner(ex, ey)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("m", [1, 4, 8, 13])
def test_gemm_inner_scaled_symmetric(ctx, m):
    rng = np.random.default_rng(m)
    v = [rand(rng, N_SMALL) for _ in range(m)]
    s = rng.choice([1.0, -0.5, 3.25], m)
    r, e = scaled_copies(ctx, v, s)
    assert np.array_equal(bits(ctx.gemm_inner_scaled(r, s, r, s)), bits(ctx.gemm_inner(e, e)))


@pytest.mark.parametrize("k,m", [(48, 8), (70, 8), (5, 16), (1, 1), (100, 3)])
@pytest.mark.parametrize("n", [N_SMALL, 2 * N_SMALL + 1])
def test_gemm_outer_scaled(ctx, k, m, n):
    rng = np.random.default_rng(k * 10 + m)
    xv = [rand(rng, n) for _ in range(k)]
    yv = [rand(rng, n) for _ in range(m)]
    xs = rng.choice([1.0, -0.5, 3.25, 0.1], k)
    ys = rng.choice([1.0, -0.5, 3.25], m)
    al = rng.uniform(-1, 1, (k, m))
    rx, ex = scaled_copies(ctx, xv, xs)
    ry, ey = scaled_copies(ctx, yv, ys)
    ctx.gemm_outer_scaled(al, rx, xs, ry, ys)
    ctx.gemm_outer(al, ex, ey)
    for a, b in zip(ry, ey):
        assert np.array_equal(bits(a.numpy()), bits(b.numpy()))
    # write-only form
    oa = [ctx.alloc(n) for _ in range(m)]
    ob = [ctx.alloc(n) for _ in range(m)]
    ctx.gemm_outer_set_scaled(al, rx, xs, oa)
    ctx.gemm_outer_set(al, ex, ob)
    for a, b in zip(oa, ob):
        assert np.array_equal(bits(a.numpy()), bits(b.numpy()))


def test_sparse_and_solution_forms_scaled(ctx):
    rng = np.random.default_rng(5)
    n, offset, m, k = N_SMALL, 1000, 8, 20
    ps = [{offset + 3: 1.0}, {offset + 7: -0.5, offset + 3: 2.0}, {offset + n - 1: 0.25},
          {5: 1.0}, {offset + 40000: 1.0, offset + 40001: -1.0}]  # {5} lies outside the shard
    xv = [rand(rng, n) for _ in range(k)]
    yv = [rand(rng, n) for _ in range(m)]
    xs = rng.choice([1.0, -0.5, 3.25], k)
    ys = rng.choice([1.0, -0.5, 3.25], m)
    rx, ex = scaled_copies(ctx, xv, xs)
    got = ctx.gemm_inner_sparse_scaled(rx, xs, ps, offset)
    assert np.array_equal(bits(got), bits(ctx.gemm_inner_sparse(ex, ps, offset)))
    pa = rng.uniform(-1, 1, (len(ps), m))
    al = rng.uniform(-1, 1, (k, m))
    # construct_solution: write-only destinations, scaled sources
    oa = [ctx.alloc(n) for _ in range(m)]
    ob = [ctx.alloc(n) for _ in range(m)]
    ctx.construct_solution_scaled(pa, ps, al, rx, xs, oa, offset)
    ctx.construct_solution(pa, ps, al, ex, ob, offset)
    for a, b in zip(oa, ob):
        assert np.array_equal(bits(a.numpy()), bits(b.numpy()))
    # block update: scaled destinations read, P then the dense sources (= scal + sparse + dense)
    for kk, pp in [(k, ps), (0, ps), (k, [])]:
        ry, ey = scaled_copies(ctx, yv, ys)
        ctx.block_update(pa[:len(pp)], pp, al[:kk], rx[:kk], xs[:kk], ry, ys, offset)
        if pp:
            ctx.gemm_outer_sparse(pa[:len(pp)], pp, ey, offset)
        if kk:
            ctx.gemm_outer(al[:kk], ex[:kk], ey)
        for a, b in zip(ry, ey):
            assert np.array_equal(bits(a.numpy()), bits(b.numpy())), (kk, len(pp))


@pytest.mark.parametrize("rank", [1, 8])
def test_synth_action_scaled(ctx, rank):
    rng = np.random.default_rng(rank)
    n, nvec = N_SMALL, 5
    xv = [rand(rng, n) for _ in range(nvec)]
    xs = np.array([1.0, -0.5, 3.25, 0.1, 1.0])
    rx, ex = scaled_copies(ctx, xv, xs)
    spec = ih.Synth(0.1, rank, 3, 0, 0.0)
    ya = [ctx.alloc(n) for _ in range(nvec)]
    yb = [ctx.alloc(n) for _ in range(nvec)]
    ctx.synth_action_scaled(rx, xs, ya, spec)
    ctx.synth_action(ex, yb, spec)
    for a, b in zip(ya, yb):
        assert np.array_equal(bits(a.numpy()), bits(b.numpy()))


@pytest.mark.parametrize("n", [1, 2, 3, 17, 1023])
def test_scaled_tails(ctx, n):
    # the element-wise tail paths (odd elements, partial windows, fewer elements than lanes)
    rng = np.random.default_rng(n)
    xv = [rand(rng, n, zeros=False) for _ in range(5)]
    yv = [rand(rng, n, zeros=False) for _ in range(3)]
    xs = np.array([-0.5, 1.0, 3.25, 0.1, -2.0])
    ys = np.array([2.5, -0.75, 1.0])
    rx, ex = scaled_copies(ctx, xv, xs)
    ry, ey = scaled_copies(ctx, yv, ys)
    assert ctx.dot_scaled(rx[0], xs[0], ry[0], ys[0]) == ctx.dot(ex[0], ey[0])
    assert np.array_equal(bits(ctx.gemm_inner_scaled(rx, xs, ry, ys)), bits(ctx.gemm_inner(ex, ey)))
    assert np.array_equal(bits(ctx.gemm_inner_scaled(rx[:1], xs[:1], ry[:2], ys[:2])),
                          bits(ctx.gemm_inner(ex[:1], ey[:2])))
    al = rng.uniform(-1, 1, (5, 3))
    ctx.gemm_outer_scaled(al, rx, xs, ry, ys)
    ctx.gemm_outer(al, ex, ey)
    for a, b in zip(ry, ey):
        assert np.array_equal(bits(a.numpy()), bits(b.numpy()))
    ctx.axpy_scaled(0.3, rx[1], xs[1], rx[2], xs[2])
    ctx.axpy(0.3, ex[1], ex[2])
    assert np.array_equal(bits(rx[2].numpy()), bits(ex[2].numpy()))
