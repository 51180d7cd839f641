"""Hot-path kernels at BASELINE.json's full sizes (N = 1e8 on one GPU: configs C3/C5; the C4 shard
N = 1.25e7 at every rank offset), checked through size-independent properties and sampled windows
against the oracle, since the oracle cannot stream 56 vectors of 1e8 doubles in seconds:

* gemm_inner is the reference's pairwise definition (util/gemm.h:267-279, testGemm.cpp:58-88):
  every entry equals the handler's own dot of that pair, and the result over [0, N) equals the sum
  of the results over two halves;
* gemm_outer / axpy (gemm.h:257-265, ArrayHandlerIterable.h:65-74) on windows at the start, the
  middle and the end of the vectors, recomputed by the oracle from the same global-index-seeded
  inputs (oracle.random_vector); an odd-length view exercises the tail path at full size;
* select / select_max_dot (select.h:28-55) bit-exact against the oracle on the whole vector;
* a C4 shard (index range [r N/8, (r+1) N/8), generated with its global offset) gives results
  bit-identical to the same range of the full vectors, and the 8 shard overlaps add up to the full
  overlap: the sharded path (DistrArray.cpp:391-401 + MPI_Allreduce) reduces to the 1-GPU one.

Tolerances: reductions |a - b| <= 64 eps sum|x_i y_i| with sum|x_i y_i| <= N (all |x|, |y| <= 1);
elementwise as tests/test_ops_gpu.py.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps
N = 100_000_000
M, K = 8, 48
SEED = 20251015
SHARDS = 8


def view(v, offset, n):
    """Non-owning view of elements [offset, offset + n) of a device vector (offset even: 16 B aligned)."""
    import subspace_hip as sh

    assert offset % 2 == 0 and offset + n <= v.n
    return sh.DeviceVector(v.ctx, n, v.ptr + 8 * offset, owner=False)


@pytest.fixture(scope="module")
def panel(ctx):
    """8 + 48 vectors of N doubles (44.8 GB of HBM), element i of vector v = oracle.random_vector."""
    xs = [ctx.alloc(N) for _ in range(M)]
    ys = [ctx.alloc(N) for _ in range(K)]
    for vid, v in enumerate(xs + ys):
        ctx.fill_random(v, SEED, vid)
    ctx.synchronize()
    yield xs, ys
    for v in xs + ys:
        v.free()
    ctx.release_cached()


def test_fill_random_windows_match_oracle(ctx, panel):
    xs, ys = panel
    for vid, v in ((0, xs[0]), (M + K - 1, ys[-1])):
        for off in (0, N // 2 + 2, N - 4096):
            got = view(v, off, 4096).numpy()
            assert np.array_equal(got, oracle.random_vector(4096, SEED, vid, off))


def test_gemm_inner_8x48_full_size_is_pairwise_dots(ctx, panel):
    xs, ys = panel
    g = ctx.gemm_inner(xs, ys)
    assert g.shape == (M, K)
    tol = 64 * EPS * N
    d = np.array([[ctx.dot(x, y) for y in ys] for x in xs])
    assert np.max(np.abs(g - d)) <= tol
    h = N // 2
    g1 = ctx.gemm_inner([view(x, 0, h) for x in xs], [view(y, 0, h) for y in ys])
    g2 = ctx.gemm_inner([view(x, h, N - h) for x in xs], [view(y, h, N - h) for y in ys])
    assert np.max(np.abs(g - (g1 + g2))) <= tol
    assert np.array_equal(ctx.gemm_inner(xs, ys), g)  # deterministic at full size
    # A 2^20-element window against the oracle on the same (downloaded) data.
    off, w = N // 3 - (N // 3) % 2, 1 << 20
    xw = [view(x, off, w) for x in xs]
    yw = [view(y, off, w) for y in ys]
    gw = ctx.gemm_inner(xw, yw)
    xh = [v.numpy() for v in xw]
    yh = [v.numpy() for v in yw]
    ref = oracle.gemm_inner(xh, yh)
    bound = 64 * EPS * (np.abs(np.array(xh)) @ np.abs(np.array(yh)).T)
    assert np.all(np.abs(gw - ref) <= bound)


def test_gemm_outer_48_to_8_full_size_windows(ctx, panel):
    xs, ys = panel
    # Destinations: 8 scratch vectors copied from xs (the panel stays intact for later tests).
    dst = [ctx.alloc(N) for _ in range(M)]
    for d, x in zip(dst, xs):
        ctx.copy(d, x)
    al = np.random.default_rng(3).uniform(-1, 1, (K, M))
    ctx.gemm_outer(al, ys, dst)
    w = 8192
    for off in (0, N // 2 + 2, N - w):
        src = [oracle.random_vector(w, SEED, M + i, off) for i in range(K)]
        old = [oracle.random_vector(w, SEED, j, off) for j in range(M)]
        ref = oracle.gemm_outer(al, src, old)
        for j in range(M):
            got = view(dst[j], off, w).numpy()
            terms = np.abs(old[j]) + np.abs(al[:, j]) @ np.abs(np.array(src))
            assert np.all(np.abs(got - ref[j]) <= 4 * K * EPS * terms)
    # Odd length at full size: the last element goes through the kernel's tail path.
    for d, x in zip(dst, xs):
        ctx.copy(d, x)
    odd = N - 1
    ctx.gemm_outer(al, [view(y, 0, odd) for y in ys], [view(d, 0, odd) for d in dst])
    e = odd - 1
    for j in range(M):
        tail = view(dst[j], N - 2, 2).numpy()
        v = oracle.random_vector(1, SEED, j, e)[0]
        for i in range(K):
            v = v + al[i, j] * oracle.random_vector(1, SEED, M + i, e)[0]
        assert abs(tail[0] - v) <= 4 * K * EPS * (abs(v) + K)
        assert tail[1] == oracle.random_vector(1, SEED, j, N - 1)[0]  # outside the view: untouched
    for d in dst:
        d.free()


def test_axpy_and_norm_full_size(ctx, panel):
    xs, ys = panel
    y = ctx.alloc(N)
    ctx.copy(y, ys[0])
    ctx.axpy(-0.375, xs[1], y)
    for off in (0, N // 2 + 2, N - 4096):
        ref = oracle.axpy(-0.375, oracle.random_vector(4096, SEED, 1, off), oracle.random_vector(4096, SEED, M, off))
        np.testing.assert_allclose(view(y, off, 4096).numpy(), ref, rtol=2 * EPS, atol=4 * EPS)
    h = N // 2
    nn = ctx.dot(y, y)
    assert abs(nn - (ctx.dot(view(y, 0, h), view(y, 0, h)) + ctx.dot(view(y, h, h), view(y, h, h)))) <= 64 * EPS * nn
    y.free()


@pytest.mark.parametrize("mode", ["min", "max", "abs"])
def test_select_full_size_bit_exact(ctx, panel, mode):
    xs, _ = panel
    host = xs[2].numpy()
    nsel = 16
    kw = {"min": {}, "max": {"max": True}, "abs": {"max": True, "ignore_sign": True}}[mode]
    gi, gv = ctx.select(xs[2], nsel, **kw)
    ri, rv = oracle.select(host, nsel, **kw)
    assert np.array_equal(np.asarray(gi), np.asarray(ri))
    assert np.array_equal(np.asarray(gv), np.asarray(rv))


def test_select_max_dot_full_size_bit_exact(ctx, panel):
    xs, ys = panel
    gi, gv = ctx.select_max_dot(xs[3], ys[3], 16)
    ri, rv = oracle.select_max_dot(xs[3].numpy(), ys[3].numpy(), 16)
    assert np.array_equal(np.asarray(gi), np.asarray(ri))
    assert np.array_equal(np.asarray(gv), np.asarray(rv))


def test_c4_shards_reduce_to_the_full_overlap(ctx, panel):
    """Config C4's shards on one GPU: rank r generates its range with its global offset."""
    xs, ys = panel
    full = ctx.gemm_inner(xs, ys)
    ns = N // SHARDS
    total = np.zeros((M, K))
    for r in range(SHARDS):
        off = r * ns
        sx = [ctx.alloc(ns) for _ in range(M)]
        sy = [ctx.alloc(ns) for _ in range(K)]
        for vid, v in enumerate(sx + sy):
            ctx.fill_random(v, SEED, vid, off)
        g = ctx.gemm_inner(sx, sy)
        # The shard's own vectors and the same range of the full vectors: same data, same result.
        assert np.array_equal(g, ctx.gemm_inner([view(x, off, ns) for x in xs], [view(y, off, ns) for y in ys]))
        assert ctx.dot(sx[0], sy[0]) == ctx.dot(view(xs[0], off, ns), view(ys[0], off, ns))
        total += g  # the allreduce, in rank order
        for v in sx + sy:
            v.free()
    assert np.max(np.abs(total - full)) <= 64 * EPS * N
