"""One rank of a multi-process check of the sharded path (launched by tests/test_distributed*.py).

  --comm gloo : launched by `torch.distributed.run`; reductions go through a gloo process group
                (subspace_hip.TorchHostComm).  torch is imported BEFORE the HIP library so the
                process holds one HIP runtime.
  --comm hub  : launched as plain subprocesses (RANK, WORLD_SIZE, SSP_HUB_PORT in the env);
                reductions go through subspace_hip.HubComm (stdlib sockets, no torch).

Cases:
  reductions  (CPU) oracle shard pieces + the product's host exchange + ssp_select_merge
  gpu_ops     (GPU) every reducing op of libsubspace_hip.so on shards, host communicator attached
  gpu_solver  (GPU) Davidson / DIIS on sharded HBM vectors vs the single-rank CPU reference path
  gpu_traces  (GPU) the committed BASELINE-size traces (C4 shape, C2, C5) on shards

Exit status 0 = every assertion held on this rank.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "iterative-solver_amd"), os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

EPS = 2.220446049250313e-16


def make_comm(kind):
    if kind == "gloo":
        import torch.distributed as dist  # first: one HIP runtime in this process

        dist.init_process_group("gloo")
        import subspace_hip as sh

        return sh.TorchHostComm()
    import subspace_hip as sh

    return sh.HubComm(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), "127.0.0.1",
                      int(os.environ["SSP_HUB_PORT"]))


def attach(ctx, comm):
    """The rank transport under test: the host communicator itself, or (SSP_TEST_TRANSPORT=p2p) the
    peer-memory communicator, whose id rank 0 makes and the hub distributes."""
    import subspace_hip as sh

    if os.environ.get("SSP_TEST_TRANSPORT") == "p2p" and comm.nranks > 1:
        uid = comm.allgather(sh.Context.p2p_unique_id() if comm.rank == 0 else bytes(128))[0]
        ctx.attach_p2p(comm.nranks, comm.rank, uid)
    else:
        ctx.attach_host_comm(comm)


def case_reductions(comm):
    import numpy as np

    import oracle
    import subspace_hip as sh

    rank, world = comm.rank, comm.nranks
    for n in (1, 3, 1001, 20_000):
        m, k, seed = 3, 5, 20251015
        off, ln = sh.shard_range(n, world, rank)
        full = [oracle.random_vector(n, seed, v) for v in range(m + k)]
        xs = [v[off:off + ln] for v in full]
        # gemm_inner: rank-local block summed over ranks through the allreduce callback.
        buf = np.ascontiguousarray((oracle.gemm_inner(xs[:m], xs[m:]) if ln else np.zeros((m, k))).ravel())
        assert comm.allreduce_cb(buf.ctypes.data_as(sh.PD), buf.size, None) == 0
        terms = np.abs(np.stack(full[:m])) @ np.abs(np.stack(full[m:])).T
        assert np.all(np.abs(buf.reshape(m, k) - oracle.gemm_inner(full[:m], full[m:])) <= 64 * EPS * terms + 1e-300)
        # sparse dot: P entries filtered to the shard range (DistrArray.cpp:419-465), then summed.
        pidx = np.unique(np.random.default_rng(seed).integers(0, n, 50))
        pval = np.linspace(-1, 1, pidx.size)
        sel = (pidx >= off) & (pidx < off + ln)
        d = np.array([oracle.sparse_dot(xs[0], pidx[sel] - off, pval[sel]) if ln else 0.0])
        assert comm.allreduce_cb(d.ctypes.data_as(sh.PD), 1, None) == 0
        assert abs(d[0] - oracle.sparse_dot(full[0], pidx, pval)) <= 1e-13 * np.sum(np.abs(pval))
        # select: per-rank best n all-gathered as raw bytes, merged identically on every rank.
        nsel = min(9, n)
        li, lv = oracle.select(xs[1], min(nsel, ln)) if ln else (np.zeros(0, np.int64), np.zeros(0))
        li = li + off
        cnts = np.zeros(world, dtype=np.uint64)
        cnt = np.array([li.size], dtype=np.uint64)
        assert comm.allgather_cb(cnt.ctypes.data, cnts.ctypes.data, 8, None) == 0
        si, sv = np.zeros(nsel, np.uint64), np.zeros(nsel)
        si[:li.size], sv[:lv.size] = li, lv
        gi, gv = np.zeros(nsel * world, np.uint64), np.zeros(nsel * world)
        assert comm.allgather_cb(si.ctypes.data, gi.ctypes.data, 8 * nsel, None) == 0
        assert comm.allgather_cb(sv.ctypes.data, gv.ctypes.data, 8 * nsel, None) == 0
        parts = [(gi[r * nsel:r * nsel + int(cnts[r])], gv[r * nsel:r * nsel + int(cnts[r])]) for r in range(world)]
        mi, mv = sh.select_merge(parts, nsel)
        ri, rv = oracle.select(full[1], nsel)
        assert np.array_equal(mi, ri) and np.array_equal(mv, rv), (mi, ri, mv, rv)


def case_gpu_ops(comm):
    import numpy as np

    import oracle
    import subspace_hip as sh

    rank, world = comm.rank, comm.nranks
    ctx = sh.Context(0)
    attach(ctx, comm)
    assert (ctx.lib.ssp_ctx_rank(ctx.handle), ctx.lib.ssp_ctx_nranks(ctx.handle)) == (rank, world)
    # 4097 on 2 ranks: shards of 2049 and 2048 elements, either side of the default exact_max -- one rank
    # takes the bandwidth kernels, the other the reference's arithmetic, in the same result layout
    for n in (5, 1003, 4097, 100_003):
        off, ln = sh.shard_range(n, world, rank)
        rng = np.random.default_rng(n)
        X = rng.uniform(-1, 1, (6, n))
        X[3] = rng.integers(-3, 4, n)  # ties for select
        xs = [ctx.upload(np.ascontiguousarray(v[off:off + ln])) for v in X]
        tol = lambda terms: 64 * EPS * terms + 1e-300  # noqa: E731
        g = ctx.dot(xs[0], xs[1])
        assert abs(g - oracle.dot(X[0], X[1])) <= tol(np.sum(np.abs(X[0] * X[1])))
        M = ctx.gemm_inner(xs[:2], xs[2:])
        terms = np.abs(X[:2]) @ np.abs(X[2:]).T
        assert np.all(np.abs(M - oracle.gemm_inner(list(X[:2]), list(X[2:]))) <= tol(terms))
        # m > k: the bandwidth kernels put the shorter side on the rows (a transposed result)
        M = ctx.gemm_inner(xs[:4], xs[4:])
        terms = np.abs(X[:4]) @ np.abs(X[4:]).T
        assert np.all(np.abs(M - oracle.gemm_inner(list(X[:4]), list(X[4:]))) <= tol(terms)), (n, M)
        assert len(set(ctx.allgather_bytes(M.tobytes()))) == 1  # every rank received the same sums
        for mx, ig in ((False, False), (True, False), (False, True)):
            nsel = min(7, n)
            gi, gv = ctx.select(xs[3], nsel, max=mx, ignore_sign=ig, offset=off)
            ri, rv = oracle.select(X[3], nsel, max=mx, ignore_sign=ig)
            assert np.array_equal(gi, ri) and np.array_equal(gv, rv), (mx, ig, gi, ri)
        gi, gv = ctx.select_max_dot(xs[3], xs[4], min(5, n), offset=off)
        ri, rv = oracle.select_max_dot(X[3], X[4], min(5, n))
        assert np.array_equal(gi, ri) and np.allclose(gv, rv, rtol=0, atol=0)
        pidx = np.unique(rng.integers(0, n, 40))
        pval = np.linspace(-2, 2, pidx.size)
        sd = ctx.sparse_dot(xs[0], pidx, pval, offset=off)
        assert abs(sd - oracle.sparse_dot(X[0], pidx, pval)) <= 1e-13 * np.sum(np.abs(pval))
        # elementwise op with global indices: sparse axpy lands only in the owning shard
        ctx.sparse_axpy(0.5, pidx, pval, xs[5], offset=off)
        assert np.array_equal(ctx.download(xs[5]), oracle.sparse_axpy(0.5, pidx, pval, X[5])[off:off + ln])
        # synthetic action: a rank x nvec reduction across shards
        y = ctx.alloc(ln)
        ctx.synthetic_action([xs[0]], [y], 0.1, 3, 11, offset=off)
        ref = oracle.synthetic_action(X[0], 0.1, 3, 11)[off:off + ln]
        assert np.allclose(ctx.download(y), ref, rtol=1e-12, atol=1e-9)
    # The fused passes' reductions (transform with its pair dots / self-dots, precondition with its
    # self-dots) on shards either side of exact_max (4097: 2049 / 2048 on 2 ranks) and with a rank
    # holding no element (n = 1): whichever branch a rank's shard takes, every rank posts a collective
    # of the same length (a mismatch hangs RCCL or fails the p2p exchange).
    for n in (1, 4097, 100_003):
        off, ln = sh.shard_range(n, world, rank)
        rng = np.random.default_rng(n + 7)
        m = 3
        X = rng.uniform(-1, 1, (m, n))
        dvals = 2.0 + np.arange(n, dtype=np.float64)
        shift = np.array([0.25, 0.5, 0.75])
        T = np.eye(m) + 0.1 * rng.uniform(-1, 1, (m, m))
        up = lambda v: ctx.upload(np.ascontiguousarray(v[off:off + ln]))  # noqa: E731
        xs = [up(v) for v in X]
        G = ctx.transform_gram(T, xs)  # x_j <- sum_i t(i, j) x_i, then the Gram matrix
        Y = T.T @ X
        assert np.all(np.abs(G - Y @ Y.T) <= 1e-12 * (np.abs(Y) @ np.abs(Y).T) + 1e-300), (n, G)
        nr = ctx.transform_norms(T, xs)
        Y = T.T @ Y
        ref = np.einsum("ij,ij->i", Y, Y)
        assert np.all(np.abs(nr - ref) <= 1e-12 * ref), (n, nr, ref)
        pv = [up(v) for v in X]
        pn = ctx.precondition_norms(pv, up(dvals), shift)
        P = X / ((dvals[None, :] - shift[:, None]) + 1e-15)
        ref = np.einsum("ij,ij->i", P, P)
        assert np.all(np.abs(pn - ref) <= 1e-12 * ref), (n, pn, ref)
        assert len(set(ctx.allgather_bytes(np.concatenate([G.ravel(), nr, pn]).tobytes()))) == 1
    ctx.close()


def case_gpu_solver(comm):
    import numpy as np

    import itsolv_hbm as ih
    import oracle
    import subspace_hip as sh

    rank, world = comm.rank, comm.nranks
    ctx = sh.Context(0)
    attach(ctx, comm)
    n, rho, seed = 100_003, 0.1, 20251015
    _, nl = sh.shard_range(n, world, rank)
    for rk, nroot, np_ in ((1, 4, 0), (4, 4, 8)):
        kw = dict(nroots=nroot, max_p=np_, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
        g = ih.davidson_synthetic(ctx, n, rho, rk, seed, n_local=nl, **kw)
        c = oracle.davidson_synthetic(n, rho, rk, seed, **kw)
        assert g["converged"] and c["converged"]
        assert g["iterations"] == c["iterations"], (g["iterations"], c["iterations"])
        scale = np.maximum(np.abs(c["eigenvalues"]), 1.0)
        assert np.all(np.abs(g["eigenvalues"] - c["eigenvalues"]) <= 1e-10 * scale)
        # every rank holds the same subspace results
        ev = comm.allreduce(np.asarray(g["eigenvalues"])) / world
        assert np.array_equal(ev, np.asarray(g["eigenvalues"]))
    kw = dict(convergence_threshold=1e-8, max_size_qspace=6)
    g = ih.diis_synthetic(ctx, 3000, 0.01, 3, 3, n_local=sh.shard_range(3000, world, rank)[1], **kw)
    c = oracle.diis_synthetic(3000, 0.01, 3, 3, **kw)
    assert g["converged"] and c["converged"] and g["iterations"] == c["iterations"]
    ctx.close()


# SSP_TRACES_FULL selects the full-size traces: BASELINE C4 (N = 1e8, 8 roots + P 16) or C5 (DIIS, N = 1e8)
FULL_TRACES = {"C4": ("C3_n1e8_rank8",), "C5": ("C5_n1e8",)}


def case_gpu_traces(comm):
    """North-star traces on shards: the C4 shape (8 roots + P 16, rank-8 H, N = 1e7), C2 and C5 (the
    well-posed DIIS instance, and the chaotic round-1 instance's fixed-length descent), sharded over
    this world on HBM, against the committed per-iteration traces of the single-rank reference CPU
    path (tests/golden/traces.json) under the same bar as the single-GPU runs
    (trace_check.assert_trace)."""
    import numpy as np

    import itsolv_hbm as ih
    import subspace_hip as sh
    from trace_check import EIG_REL, T, assert_trace, run_case, solution_target

    rank, world = comm.rank, comm.nranks
    ctx = sh.Context(0)
    attach(ctx, comm)
    names = ("C3_n1e7_rank8", "C2_rank8", "C5_n1e7", "C5x_n1e7_traj12", "RS_n2e21_p16", "RS_n2e21_rho1")
    if os.environ.get("SSP_TRACES_FULL"):
        names = FULL_TRACES[os.environ["SSP_TRACES_FULL"]]
    for name in names:
        ref = T[name]
        c = ref["case"]
        nl = sh.shard_range(c["n"], world, rank)[1]
        g = run_case(ih, ctx, ref, n_local=nl, solutions=c["kind"] == "diis")
        assert_trace(g, ref, f"{name} on {world} shards")
        if c["kind"] == "diis" and ref["converged"]:  # x = t 1 (t = 1/sqrt(N)) on every shard
            assert np.max(np.abs(g["x"] - solution_target(ref))) <= ref["options"]["convergence_threshold"], name
        if rank == 0:
            print(f"{name} on {world} shards: {g['iterations']} iterations (CPU path {ref['iterations']}), "
                  f"{g['seconds']:.3f} s", flush=True)
        if c["kind"] == "davidson":
            np.testing.assert_allclose(g["eigenvalues"], ref["eigenvalues"], rtol=EIG_REL, atol=0)
    ctx.close()


def case_gpu_exact_mpi(comm):
    """Rank-order sums, bit for bit: on shards of at most ssp_ctx_set_exact_max elements every rank
    computes in the reference's arithmetic and the transport adds the ranks' partials in rank order
    (peer memory, host hub) -- one valid association of the reference's MPI_Allreduce -- so a sharded
    solve over P ranks must reproduce the CPU path run with its dots summed that way
    (tests/golden/mpi_traces.json, make_traces.py --mpi-golden): every iteration count, trace value,
    eigenvalue and error to the last bit, including the DIIS case whose step count the reference
    itself changes with the association (rank order: 13, 13, 32, 12, 56 steps at P = 1, 2, 3, 4, 8;
    MPICH's: 13, 13, 32, 46, 32 -- tests/golden/mpich_traces.json, tests/test_mpi_bridge*.py)."""
    import json

    import numpy as np

    import itsolv_hbm as ih
    import subspace_hip as sh

    rank, world = comm.rank, comm.nranks
    gold = json.load(open(os.path.join(HERE, "golden", "mpi_traces.json")))
    ctx = sh.Context(0)
    attach(ctx, comm)
    for name, rec in gold.items():
        if name.startswith("_"):
            continue
        c, ref = rec["case"], rec[f"mpi{world}"]
        nl = sh.shard_range(c["n"], world, rank)[1]
        fn = ih.davidson_synthetic if c["kind"] == "davidson" else ih.diis_synthetic
        g = fn(ctx, c["n"], c["rho"], c["rank"], c["seed"], n_local=nl, solutions=False, **rec["options"])
        head = f"{name} on {world} shards"
        assert (g["iterations"], g["converged"]) == (ref["iterations"], ref["converged"]), (head, g["iterations"])
        assert (g["r_creations"], g["q_creations"]) == (ref["r_creations"], ref["q_creations"]), head
        # (residual_norms: a post-solve diagnostic of the harness, summed sequentially by the oracle
        # whatever the order of its dots; not compared here)
        for f in ("eigenvalues", "errors"):
            if ref[f]:
                assert np.array_equal(np.asarray(g[f]), np.asarray(ref[f])), (head, f, g[f], ref[f])
        for f in ("eigenvalues", "errors", "nq", "nwork", "screened"):
            if len(ref["trace"][f]):
                assert np.array_equal(np.asarray(g["trace"][f]), np.asarray(ref["trace"][f])), (head, "trace", f)
        if rank == 0:
            print(f"{head}: {g['iterations']} iterations, bit-identical to the CPU path with {world}-rank rank-order sums",
                  flush=True)
    ctx.close()


def case_gpu_distr(comm):
    """The reference's distributed-array known answers (tests/distr_cases.py) on HBM shards."""
    import distr_cases
    import subspace_hip as sh

    ctx = sh.Context(0)
    attach(ctx, comm)
    distr_cases.check(ctx, sh, comm.rank, comm.nranks)
    ctx.close()


def case_gpu_peer_lost(comm):
    """Fail fast instead of hanging when a rank is lost mid-solve.  Both ranks repeat sharded Davidson
    solves (C2's shape at N = 1e7).  Host transport: rank 1 dies (os._exit) 1 s in, and rank 0's next
    reduction must fail with SSP_ERR_COMM at once (the peer's socket closes).  Peer-memory transport:
    rank 1 stops taking part after its first solve, but stays alive (so no rank frees memory another
    rank's kernel may still address); rank 0's next exchange must fail within SSP_COMM_TIMEOUT_S with
    the device-side deadline naming rank 1, and rank 1 must then see the abort too.  Returns True: no
    closing barrier (the communicator is gone)."""
    import threading
    import time

    import itsolv_hbm as ih
    import subspace_hip as sh

    rank, world = comm.rank, comm.nranks
    transport = os.environ.get("SSP_TEST_TRANSPORT", "host")
    timeout = float(os.environ["SSP_COMM_TIMEOUT_S"])
    ctx = sh.Context(0)
    attach(ctx, comm)
    n = 10_000_000
    nl = sh.shard_range(n, world, rank)[1]
    kw = dict(nroots=4, max_p=0, convergence_threshold=1e-8, max_size_qspace=24, reset_D=8)
    solve = lambda: ih.davidson_synthetic(ctx, n, 0.1, 8, 1, n_local=nl, solutions=False, **kw)  # noqa: E731
    t_lost = None
    if rank == 1:
        if transport == "host":
            threading.Timer(1.0, lambda: os._exit(17)).start()
            while True:
                solve()
        solve()
        time.sleep(timeout + 8)  # missing from rank 0's next exchange, but alive
        try:
            ctx.dot(ctx.alloc(nl), ctx.alloc(nl))
            raise AssertionError("rank 1: exchange after the abort succeeded")
        except sh.SspError as e:
            assert e.code == 5, e
            print(f"rank 1 sees the abort: {e}", flush=True)
        ctx.close()
        return True
    solve()
    t_lost = time.time()
    try:
        while True:
            solve()
            t_lost = time.time()
    except RuntimeError as e:
        dt = time.time() - t_lost
        msg = str(e)
        print(f"rank 0: error {dt:.2f} s after the last completed solve: {msg}", flush=True)
        if transport == "host":
            assert "callback failed" in msg, msg
            assert dt < 30, dt
        else:  # the device-side deadline of a reduction, or the host deadline of a gather
            assert "rank 1 did not arrive" in msg or "no completion within" in msg, msg
            assert timeout - 1 < dt < timeout + 20, dt
    # every later exchange fails at once
    t0 = time.time()
    try:
        ctx.dot(ctx.alloc(nl), ctx.alloc(nl))
        raise AssertionError("rank 0: exchange after the abort succeeded")
    except sh.SspError as e:
        assert e.code == 5 and time.time() - t0 < 1.0, e
    ctx.close()
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comm", choices=["gloo", "hub"], required=True)
    ap.add_argument("--case", choices=["reductions", "gpu_ops", "gpu_solver", "gpu_distr", "gpu_traces",
                                       "gpu_peer_lost", "gpu_exact_mpi"], required=True)
    a = ap.parse_args()
    comm = make_comm(a.comm)
    no_barrier = {"reductions": case_reductions, "gpu_ops": case_gpu_ops, "gpu_solver": case_gpu_solver,
                  "gpu_distr": case_gpu_distr, "gpu_traces": case_gpu_traces,
                  "gpu_peer_lost": case_gpu_peer_lost, "gpu_exact_mpi": case_gpu_exact_mpi}[a.case](comm)
    if no_barrier:
        print(f"rank {comm.rank}/{comm.nranks} {a.case} OK", flush=True)
        os._exit(0)  # the hub peer may be gone: no closing collective
    if a.comm == "gloo":
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    else:
        comm.barrier()
        comm.close()
    print(f"rank {comm.rank}/{comm.nranks} {a.case} OK", flush=True)


if __name__ == "__main__":
    main()
