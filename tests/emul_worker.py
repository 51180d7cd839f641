"""Runs the product's HOST code (restated solvers, HBM handlers, reverse-communication C API, the
Python bindings) over the host-memory emulation of the device ABI (oracle/ssp_emul.cpp), in a
fresh process so that no real HIP library is loaded beside it.  TEST INFRASTRUCTURE: the GPU
parity of the same code over libsubspace_hip.so is tests/test_*_gpu.py.

  python tests/emul_worker.py api              single rank: Python API + C-API loop parity
  RANK=r WORLD_SIZE=w SSP_HUB_PORT=p python tests/emul_worker.py spmd
                                               one rank of a sharded solve (socket host communicator)
  python -m torch.distributed.run --nproc-per-node 2 ... tests/emul_worker.py spmd-gloo
                                               the same over a gloo process group
Exit status 0 = every assertion held.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "iterative-solver_amd"), os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import iterative_solver  # noqa: E402
import itsolv_hbm as ih  # noqa: E402
import oracle  # noqa: E402
import subspace_hip as sh  # noqa: E402

EMUL = os.path.join(ROOT, "oracle", "build")
sh.LIB_PATH = os.path.join(EMUL, "libssp_emul.so")
ih.LIB_PATH = os.path.join(EMUL, "libitsolv_emul.so")
iterative_solver.LIB_PATH = os.path.join(EMUL, "libitsolv_emul.so")
BIG = 1.7976931348623157e308


def case_api():
    from test_python_api import RayleighQuotient
    from test_python_api_gpu import Dense, hamiltonian

    # reference python/test/test_rayleigh_quotient.py: test_diagonalize, test_nonlinear_equations
    problem = RayleighQuotient(8, 0.1)
    x, g = np.zeros([2, 8]), np.zeros([2, 8])
    s = iterative_solver.LinearEigensystem(8, 2)
    s.solve(x, g, problem, generate_initial_guess=True)
    s.solution([0, 1], x, g)
    assert np.all(s.errors < 1e-7), s.errors
    assert np.allclose(s.eigenvalues, problem.eigenvalues[:2], atol=1e-7)
    s.finalize()
    problem = RayleighQuotient(4, 0.01)
    x, g = np.zeros(4), np.zeros(4)
    x[0] = 1
    s = iterative_solver.NonLinearEquations(4)
    s.solve(x, g, problem)
    s.solution([0], x, g)
    x = x * problem.eigenvectors[0, 0] / x[0]
    assert abs(problem.residual(x, g) - problem.eigenvalues[0]) < 1e-7
    s.finalize()
    # reference test_rayleigh_quotient.py:152-215: LinearEquations through the C API
    import test_python_api_gpu as tg

    tg.test_linear_equations()
    tg.test_simple_linear_equations()
    tg.test_optimize("")
    tg.test_optimize("SD")
    # method dispatch of the C API through the SolverFactory restatement (SolverFactory.h:114-185):
    # unknown methods raise "Unimplemented method <m>", the named methods construct
    from test_python_api_gpu import check_factory_dispatch, check_instance_lifecycle, check_minimize_flag_ignored

    check_factory_dispatch()
    check_instance_lifecycle()
    check_minimize_flag_ignored()
    # RSPT (test_RSPT.cpp:191-196) through the product host code: the reference path's steps
    import rc_problems as rp

    for name in ("he", "hf"):
        h, h0 = rp.rspt_problem(name)
        ref = rp.loop_rspt(oracle.RcSolver("LinearEigensystem", h0.size, thresh=1e-8, algorithm="RSPT"), h, h0)
        s = iterative_solver.LinearEigensystem(h0.size, 1, thresh=1e-8, hermitian=True, algorithm="RSPT")
        trace = rp.loop_rspt(s, h, h0)
        assert [t[:-1] for t in trace] == [t[:-1] for t in ref], name
        for a, b in zip(trace, ref):
            assert np.max(np.abs(a[-1] - b[-1])) <= 1e-9 * max(1.0, np.max(np.abs(b[-1]))), name
        s.finalize()
    # C-API loop vs the restated solve() of the CPU reference path: same iterations
    for name, split, nroot in (("he", 0.0, 1), ("hf", 1e-8, 3), ("bh", 1e-8, 3)):
        h = hamiltonian(name, split)
        n = h.shape[0]
        cpu = oracle.davidson_dense(h, nroots=nroot, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
        s = iterative_solver.LinearEigensystem(n, nroot, thresh=1e-8, thresh_value=BIG, hermitian=True,
                                               options=f"MAX_SIZE_QSPACE={6 * nroot},RESET_D=8")
        x, g = np.zeros((nroot, n)), np.zeros((nroot, n))
        for k, i in enumerate(sorted(np.argsort(np.diag(h), kind="stable")[:nroot])):
            x[k, i] = 1.0
        s.solve(x, g, Dense(h))
        assert s.statistics()["iterations"] == cpu["iterations"], (name, s.statistics(), cpu["iterations"])
        assert np.max(np.abs(s.eigenvalues - cpu["eigenvalues"])) < 1e-10
        s.finalize()


def case_spmd(gloo=False):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if gloo:
        import torch.distributed as dist  # no HIP runtime in this process: the emulator has none

        dist.init_process_group("gloo")
        comm = sh.TorchHostComm()
    else:
        comm = sh.HubComm(rank, world, "127.0.0.1", int(os.environ["SSP_HUB_PORT"]))
    ctx = sh.Context(0)
    ctx.attach_host_comm(comm)
    n = 20_011
    _, nl = sh.shard_range(n, world, rank)
    # the whole Davidson solve, sharded: each rank holds its index range of every vector
    for rk, nroot, np_ in ((1, 3, 0), (4, 4, 8)):
        kw = dict(nroots=nroot, max_p=np_, convergence_threshold=1e-8, max_size_qspace=6 * nroot, reset_D=8)
        got = ih.davidson_synthetic(ctx, n, 0.1, rk, 7, n_local=nl, **kw)
        ref = oracle.davidson_synthetic(n, 0.1, rk, 7, **kw)
        assert got["converged"] and ref["converged"]
        assert got["iterations"] == ref["iterations"], (got["iterations"], ref["iterations"])
        assert np.max(np.abs(got["eigenvalues"] - ref["eigenvalues"])) <= 1e-10 * np.max(np.abs(ref["eigenvalues"]))
    got = ih.diis_synthetic(ctx, 3000, 0.01, 3, 3, n_local=sh.shard_range(3000, world, rank)[1],
                            convergence_threshold=1e-8, max_size_qspace=6)
    ref = oracle.diis_synthetic(3000, 0.01, 3, 3, convergence_threshold=1e-8, max_size_qspace=6)
    assert got["converged"] and got["iterations"] == ref["iterations"]
    # the reverse-communication C API on shards (sync=True gathers full vectors on every rank)
    m = np.ones((60, 60)) + np.diag(3.0 * np.arange(1, 61))
    iterative_solver.use_context(ctx)
    rng = [0, 0]
    s = iterative_solver.LinearEigensystem(60, 3, range=rng, thresh=1e-8, thresh_value=BIG, hermitian=True)
    assert tuple(rng) == sh.shard_range(60, world, rank)[0:1] + (sum(sh.shard_range(60, world, rank)),)
    x, g = np.zeros((3, 60)), np.zeros((3, 60))
    x[0, 0] = x[1, 1] = x[2, 2] = 1
    d = np.diag(m)
    nwork = 3
    for _ in range(60):
        g[:nwork] = x[:nwork] @ m
        nwork = s.add_vector(x[:nwork], g[:nwork])
        ev = s.working_set_eigenvalues(nwork)
        for k in range(nwork):
            g[k] = g[k] / ((d - ev[k]) + 1e-15)
        nwork = s.end_iteration(x, g)
        if nwork == 0:
            break
    assert nwork == 0
    assert np.allclose(s.eigenvalues, np.linalg.eigvalsh(m)[:3], atol=1e-8, rtol=0)
    s.finalize()
    if gloo:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    else:
        comm.barrier()
        comm.close()


def case_c4(gloo=False):
    """BASELINE configs C4 / C5 at world size 8 (socket host communicator): the sharded Davidson with
    C3/C4's options and the sharded DIIS with C5's, at N = 16_003 (shards 2000-2001 long), against the
    independent restatement (oracle/itsolv_np.py) and the unsharded CPU path (rank 0 checks): same
    steps."""
    import itsolv_np

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    comm = sh.HubComm(rank, world, "127.0.0.1", int(os.environ["SSP_HUB_PORT"]))
    ctx = sh.Context(0)
    ctx.attach_host_comm(comm)
    n = 16_003
    _, nl = sh.shard_range(n, world, rank)
    kw = dict(nroots=8, max_p=16, convergence_threshold=1e-8, max_size_qspace=48, reset_D=8)
    got = ih.davidson_synthetic(ctx, n, 0.1, 8, 1, n_local=nl, **kw)
    c5 = dict(convergence_threshold=1e-8, max_size_qspace=6)
    got5 = ih.diis_synthetic(ctx, n, 0.01, 3, 3, n_local=nl, **c5)
    comm.barrier()
    comm.close()
    if rank:
        return
    ind = itsolv_np.Davidson(8, 1e-8, max_size_qspace=48, reset_D=8, max_p=16).solve(
        itsolv_np.SyntheticProblem(n, 0.1, 8, 1))
    ref = oracle.davidson_synthetic(n, 0.1, 8, 1, solutions=False, **kw)
    print("c4: sharded", got["iterations"], "iterations; independent", ind["iterations"], "; cpu", ref["iterations"],
          "; c5 sharded", got5["iterations"], flush=True)
    for other in (ind, ref):
        assert got["converged"] == other["converged"] and got["iterations"] == other["iterations"]
        assert got["r_creations"] == other["r_creations"]
        assert [int(x) for x in got["trace"]["nq"]] == [int(x) for x in other["trace"]["nq"]]
        assert [int(x) for x in got["trace"]["nwork"]] == [int(x) for x in other["trace"]["nwork"]]
        assert np.max(np.abs(got["eigenvalues"] - np.asarray(other["eigenvalues"])[:8])) <= 1e-10 * 9
    got = got5
    ind = itsolv_np.DIIS(1e-8, max_size_qspace=6).solve(itsolv_np.SyntheticProblem(n, 0.01, 3, 3))
    assert got["converged"] and ind["converged"] and got["iterations"] == ind["iterations"]
    e = [x[0] for x in got["trace"]["errors"][:5]]
    ei = [x[0] for x in ind["trace"]["errors"][:5]]
    assert np.allclose(e, ei, rtol=1e-4, atol=0), (e, ei)


def case_rs_traces():
    """The near-dependent trace cases (traces.json RS_*: N = 2^21, the redundancy screen fires) through
    the product's host code over the emulation: above the 2^20 threshold, so the fused solver passes
    (one-pass self-orthonormalisation, batched overlap rows, residuals with their norms, block
    Gram-Schmidt) run, with the emulation's arithmetic set by argv[2] = "sum_order,fma" (0,0: the
    reference's sequential uncontracted loops; 1,1: 8-lane sums and fma, as a GPU rounds).  Full trace
    bar against the committed CPU-path traces (tests/trace_check.py)."""
    import ctypes

    from trace_check import T, assert_trace, run_case

    so, fma = (int(v) for v in sys.argv[2].split(","))
    lib = ctypes.CDLL(sh.LIB_PATH)
    assert lib.ssp_emul_set_arith(so, fma) == 0
    ctx = sh.Context(0)
    for name in ("RS_n2e21_p16", "RS_n2e21_rho1"):
        ref = T[name]
        g = run_case(ih, ctx, ref, solutions=False)
        assert g["redundant_params"] > 0, name
        assert_trace(g, ref, f"{name} (emulated device, arith {so},{fma})")
        np.testing.assert_allclose(g["eigenvalues"], ref["eigenvalues"], rtol=1e-10, atol=0)
        print(name, g["iterations"], "iterations,", g["redundant_params"], "redundant", flush=True)
    ctx.close()


def case_devsel():
    """The reference C API's instances take the device of the node-local rank the launcher exported
    (iterative_solver_c.cpp default_device) modulo the visible device count; argv[2] = expected."""
    import ctypes

    s = iterative_solver.LinearEigensystem(8, 1)
    got = ctypes.CDLL(sh.LIB_PATH).ssp_emul_last_device()
    s.finalize()
    assert got == int(sys.argv[2]), (got, sys.argv[2])


def case_distr():
    """The reference's distributed-array known answers (tests/distr_cases.py) at this world size."""
    import distr_cases

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    comm = sh.HubComm(rank, world, "127.0.0.1", int(os.environ["SSP_HUB_PORT"]))
    ctx = sh.Context(0)
    ctx.attach_host_comm(comm)
    distr_cases.check(ctx, sh, rank, world)
    comm.barrier()
    comm.close()


def case_api_record():
    """tests/api_cases.py on the CPU path (the product's host code over the emulation, the reference's
    arithmetic), written to argv[2] as JSON for tests/test_python_api_gpu.py to compare bit for bit."""
    import json

    import api_cases

    json.dump(api_cases.run_all(iterative_solver), open(sys.argv[2], "w"))


def case_exact_mpi():
    """The bit-for-bit check of rank-order sums that the GPU runs (dist_worker case_gpu_exact_mpi),
    through the product's host code over the emulation: sequential sums on each rank, the partials
    added in rank order by the socket host communicator."""
    import dist_worker

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    comm = sh.HubComm(rank, world, "127.0.0.1", int(os.environ["SSP_HUB_PORT"]))
    dist_worker.case_gpu_exact_mpi(comm)
    comm.barrier()
    comm.close()


if __name__ == "__main__":
    {"api": case_api, "spmd": case_spmd, "spmd-gloo": lambda: case_spmd(gloo=True), "c4": case_c4, "distr": case_distr,
     "devsel": case_devsel, "rs_traces": case_rs_traces, "exact_mpi": case_exact_mpi, "api_record": case_api_record}[sys.argv[1]]()
    print(f"{sys.argv[1]} OK", flush=True)
