"""The reference's distributed-array known answers on the product's sharded ops (every rank holds its
index range; reductions and selections go through the context's communicator).  Shared by
tests/emul_worker.py (host emulation, world sizes 1-4) and tests/dist_worker.py (MI355X, two ranks on
the one device through the host communicator).

  testDistrArray.h:110-131     select_max_dot: x = global index, y = 1, n = 5 -> {25..29: 25..29}
  testDistrArray.h:319-399     min_loc_n / reversed / max_n / min_abs_n / max_abs_n over dim 30
                               (the ArrayHandler interface's select(n, x, max, ignore_sign),
                               ArrayHandler.h:219-222, returns the index-ordered map)
  testDistrArray.h:526-588     axpy, axpy_map, dot_array, dot_map (collective linear algebra)
  testArrayHandlerDistrSparse.cpp:23-62   sparse axpy and dot over dim 20 with
                               {1: 1, 3: 2, 6: 3, 11: 4}: dot = 0.5 (1 + 2 + 3 + 4) = 5
  testDistribution.cpp:58-62   make_distribution_spread_remainder(11, 3) = {0, 4, 8, 11}
  testGemm.cpp:228-257, :290-326, :463-497   distrsparse_inner, distr_outer, distrsparse_outer: the
                               gemm forms equal the handler's pairwise dot / axpy loops (x_i = iota
                               from i + 0.5, sparse {1: i+1, 3: i+2, 6: i+3, 9: i+4}, alpha = iota
                               from 1, n = dim = 10)
"""
import numpy as np


def check(ctx, sh, rank, world):
    def shard(dim):
        return sh.shard_range(dim, world, rank)

    def upload_range(values):
        off, ln = shard(len(values))
        return ctx.upload(np.ascontiguousarray(values[off:off + ln], dtype=np.float64)), off

    # testDistribution.cpp:58-62
    assert [sh.shard_range(11, 3, r)[0] for r in range(3)] + [11] == [0, 4, 8, 11]

    dim = 30
    # select_max_dot (testDistrArray.h:110-131)
    x, off = upload_range(np.arange(dim, dtype=np.float64))
    y, _ = upload_range(np.ones(dim))
    idx, val = ctx.select_max_dot(x, y, 5, offset=off)
    assert dict(zip(idx.tolist(), val.tolist())) == {i: float(i) for i in range(25, 30)}, (idx, val)

    # min_loc_n / max_n / min_abs_n / max_abs_n (testDistrArray.h:319-399): values 0..29
    idx, _ = ctx.select(x, 10, max=False, offset=off)
    assert idx.tolist() == list(range(10)), idx
    idx, _ = ctx.select(x, 10, max=True, offset=off)
    assert idx.tolist() == list(range(20, 30)), idx
    xr, _ = upload_range(np.arange(dim, dtype=np.float64)[::-1].copy())  # min_loc_n_reverse
    idx, _ = ctx.select(xr, 10, max=False, offset=off)
    assert idx.tolist() == list(range(20, 30)), idx
    alt = np.arange(dim, dtype=np.float64)
    alt[1::2] *= -1
    xa, _ = upload_range(alt)
    idx, _ = ctx.select(xa, 10, max=False, ignore_sign=True, offset=off)
    assert idx.tolist() == list(range(10)), idx
    idx, _ = ctx.select(xa, 10, max=True, ignore_sign=True, offset=off)
    assert idx.tolist() == list(range(20, 30)), idx

    # axpy (testDistrArray.h:526-540): a = alpha + scale * beta everywhere, b unchanged
    alpha, beta, scale = 1.5, -0.75, -3.0
    a, _ = upload_range(np.full(dim, alpha))
    b, _ = upload_range(np.full(dim, beta))
    ctx.axpy(scale, b, a)
    assert np.all(a.numpy() == alpha + scale * beta) and np.all(b.numpy() == beta)

    # axpy_map / dot_map / dot_array (testDistrArray.h:542-588)
    sparse = {1: 1.0, 3: 2.0, 6: 3.0, 11: 4.0, 29: -2.5}
    pidx, pval = np.array(list(sparse)), np.array(list(sparse.values()))
    a, _ = upload_range(np.full(dim, alpha))
    ctx.sparse_axpy(5.0, pidx, pval, a, offset=off)
    ref = np.full(dim, alpha)
    ref[pidx] += 5.0 * pval
    o, ln = shard(dim)
    assert np.array_equal(a.numpy(), ref[o:o + ln])
    range_alpha = 0.25 * np.arange(1, dim + 1)
    range_beta = -1.0 + 0.5 * np.arange(dim)
    ra, _ = upload_range(range_alpha)
    rb, _ = upload_range(range_beta)
    assert ctx.dot(ra, rb) == np.inner(range_alpha, range_beta)  # exact: small integers / quarters
    assert ctx.sparse_dot(ra, pidx, pval, offset=off) == sum(range_alpha[i] * v for i, v in sparse.items())

    # testArrayHandlerDistrSparse.cpp:23-62 over dim 20
    d20 = 20
    m20 = {1: 1.0, 3: 2.0, 6: 3.0, 11: 4.0}
    i20, v20 = np.array(list(m20)), np.array(list(m20.values()))
    y20, off20 = upload_range(np.full(d20, 0.5))
    ctx.sparse_axpy(2.0, i20, v20, y20, offset=off20)
    ref = np.full(d20, 0.5)
    ref[i20] += 2.0 * v20
    o, ln = shard(d20)
    assert np.array_equal(y20.numpy(), ref[o:o + ln])
    x20, _ = upload_range(np.full(d20, 0.5))
    assert ctx.sparse_dot(x20, i20, v20, offset=off20) == 0.5 + 0.5 * 2.0 + 0.5 * 3.0 + 0.5 * 4.0

    # testGemm.cpp distrsparse_inner / distr_outer / distrsparse_outer (n = dim = 10)
    n = dim = 10
    vx = [np.arange(dim) + i + 0.5 for i in range(n)]
    my = [{1: i + 1.0, 3: i + 2.0, 6: i + 3.0, 9: i + 4.0} for i in range(n)]
    cx = [upload_range(v)[0] for v in vx]
    off = shard(dim)[0]
    g = ctx.gemm_inner_sparse(cx, my, offset=off)
    ref = np.array([[sum(vx[i][k] * v for k, v in my[j].items()) for j in range(n)] for i in range(n)])
    pair = np.array([[ctx.sparse_dot(cx[i], list(my[j]), list(my[j].values()), offset=off) for j in range(n)]
                     for i in range(n)])
    assert np.all(np.abs(g - pair) <= 4 * np.finfo(float).eps * np.abs(ref)), np.max(np.abs(g - pair))
    assert np.all(np.abs(g - ref) <= 4 * np.finfo(float).eps * np.abs(ref))
    alpha = np.arange(1, n * n + 1, dtype=np.float64).reshape(n, n)
    cy = [upload_range(v)[0] for v in vx]
    cz = [upload_range(v)[0] for v in vx]
    ctx.gemm_outer(alpha, cx, cy)  # cy[j] += sum_i alpha(i, j) cx[i]
    for i in range(n):
        for j in range(n):
            ctx.axpy(alpha[i, j], cx[i], cz[j])
    for j in range(n):
        assert np.array_equal(cy[j].numpy(), cz[j].numpy())  # the reference's summation order per destination
    cx = [upload_range(v)[0] for v in vx]
    cy = [upload_range(v)[0] for v in vx]
    ctx.gemm_outer_sparse(alpha, my, cx, offset=off)  # cx[j] += sum_i alpha(i, j) my[i]
    for i in range(n):
        for j in range(n):
            ctx.sparse_axpy(alpha[j, i], list(my[j]), list(my[j].values()), cy[i], offset=off)
    o, ln = shard(dim)
    for i in range(n):
        full = vx[i].copy()
        for j in range(n):
            for k, v in my[j].items():
                full[k] += alpha[j, i] * v
        assert np.allclose(cx[i].numpy(), cy[i].numpy(), rtol=4 * np.finfo(float).eps, atol=0)
        assert np.allclose(cx[i].numpy(), full[o:o + ln], rtol=8 * np.finfo(float).eps, atol=0)
