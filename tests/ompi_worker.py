"""One process with a one-rank Open MPI ABI stand-in (tests/fake_ompi/fake_ompi.c, test infrastructure)
loaded RTLD_GLOBAL before the product, as an Open MPI caller would have it: the fcomm bridge must take
its Open MPI branch (iterative-solver_amd/host/mpi_bridge.cpp Impl<void*>: handles are object
addresses, MPI_Comm_f2c / _c2f are functions, MPI_IN_PLACE is (void*)1).  Launched by
tests/test_ompi_bridge.py.

  python ompi_worker.py LIBFAKE capi|init

capi: MPI_Init by the caller; the reference's C-API loops with the default communicator
      (IterativeSolver_mpicomm_global() = Open MPI's Fortran MPI_COMM_WORLD, 0) take the CPU path's
      steps bit for bit; every MPI call the bridge made held to the ABI; an unknown Fortran handle is
      refused; a transport preference list falls back to MPI.
init: MPI loaded but not initialised: IterativeSolver_mpi_init / _mpi_finalize start and end it.

Over the host emulation of the device ABI (oracle/build, test infrastructure).  Exit 0 = every
assertion held.
"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "iterative-solver_amd"), os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

FAKE = C.CDLL(sys.argv[1], mode=C.RTLD_GLOBAL)
FAKE.fake_ompi_count.restype = C.c_long
FAKE.fake_ompi_count.argtypes = [C.c_char_p]
if sys.argv[2] != "init":
    assert FAKE.MPI_Init(None, None) == 0

import numpy as np  # noqa: E402

import iterative_solver  # noqa: E402
import itsolv_hbm as ih  # noqa: E402
import subspace_hip as sh  # noqa: E402

EMUL = os.path.join(ROOT, "oracle", "build")
sh.LIB_PATH = os.path.join(EMUL, "libssp_emul.so")
ih.LIB_PATH = os.path.join(EMUL, "libitsolv_emul.so")
iterative_solver.LIB_PATH = os.path.join(EMUL, "libitsolv_emul.so")
BIG = 1.7976931348623157e308
OPTS6 = "convergence_threshold=1e-8,max_size_qspace=6"


def count(what):
    return FAKE.fake_ompi_count(what.encode())


def case_capi():
    import oracle
    import rc_problems as rp

    lib = iterative_solver._load()
    lib.IterativeSolver_mpicomm_self.restype = C.c_int64
    assert lib.IterativeSolverHbmMpiActive() == 1
    # Open MPI's Fortran handles: MPI_COMM_WORLD 0, MPI_COMM_SELF 1 (MPI_Comm_c2f of the objects)
    assert iterative_solver._call("IterativeSolver_mpicomm_global") == 0
    assert lib.IterativeSolver_mpicomm_self() == 1
    c2f = count("c2f")
    assert c2f >= 2
    rng = [0, 0]
    s = iterative_solver.LinearEigensystem(7, 1, range=rng, thresh=1e-8)
    assert tuple(rng) == (0, 7)
    s.finalize()
    checked = 0
    for n, hermitian in ((7, True), (28, True), (13, False)):
        h = rp.eigen_matrix(n, non_hermiticity=0.0 if hermitian else 0.01)
        for nroot, np_ in list(rp.eigen_cases(n, hermitian))[:4]:
            opts = rp.eigen_options(n, nroot, np_, hermitian)
            ref = oracle.RcSolver("LinearEigensystem", n, nroot, thresh=1e-8, thresh_value=BIG, hermitian=hermitian,
                                  options=opts)
            rtrace, riter = rp.loop_eigen(ref, h, nroot, np_)
            got = iterative_solver.LinearEigensystem(n, nroot, thresh=1e-8, thresh_value=BIG, hermitian=hermitian,
                                                     options=opts)
            gtrace, giter = rp.loop_eigen(got, h, nroot, np_)
            head = f"eigen n={n} nroot={nroot} np={np_} (Open MPI ABI)"
            assert (gtrace, giter) == (rtrace, riter), (head, gtrace, rtrace)
            assert np.array_equal(np.asarray(got.eigenvalues), np.asarray(ref.stats()["eigenvalues"])[:nroot]), head
            assert np.array_equal(got.errors, ref.stats()["errors"]), head
            got.finalize()
            checked += 1
    for kind, optimize in (("NonLinearEquations", False), ("Optimize", True)):
        h = rp.quadratic_matrix(20, 10.0)
        ref = oracle.RcSolver(kind, 20, thresh=1e-8, options=OPTS6)
        rtrace, _ = rp.loop_quadratic(ref, h, optimize)
        got = (iterative_solver.Optimize if optimize else iterative_solver.NonLinearEquations)(20, thresh=1e-8,
                                                                                                options=OPTS6)
        gtrace, _ = rp.loop_quadratic(got, h, optimize)
        assert [t[:2] for t in gtrace] == [t[:2] for t in rtrace], kind
        assert all(np.array_equal(a[2], b[2]) for a, b in zip(gtrace, rtrace)), kind
        got.finalize()
        checked += 1
    # The attach itself (IterativeSolverHbmMpiAttach, what the Initialize calls do for a communicator of
    # several ranks): an unknown Fortran handle -- MPI_Comm_f2c gives NULL -- is refused; "p2p,mpi" and
    # "mpi" attach over the world, through the node split and the agreed outcomes.
    lib.IterativeSolverHbmMpiAttach.argtypes = [C.c_void_p, C.c_int64, C.c_char_p]
    lib.IterativeSolverHbmLastError.restype = C.c_char_p
    ctx = sh.Context(0)
    assert lib.IterativeSolverHbmMpiAttach(ctx.handle, 77, b"mpi") != 0
    assert b"is not a communicator" in lib.IterativeSolverHbmLastError()
    for transport in (b"p2p,mpi", b"mpi", b"rccl,mpi"):
        assert lib.IterativeSolverHbmMpiAttach(ctx.handle, 0, transport) == 0, lib.IterativeSolverHbmLastError()
        assert (ctx.lib.ssp_ctx_rank(ctx.handle), ctx.lib.ssp_ctx_nranks(ctx.handle)) == (0, 1)
    ctx.close()
    # the agreements went through the caller's MPI_Allreduce (in place) and MPI_Bcast with Open MPI's
    # predefined handles (one rank: the solves' own reductions need no exchange)
    assert count("allreduce") >= 3 and count("in_place") == count("allreduce") and count("bcast") >= 1, (
        count("allreduce"), count("in_place"), count("bcast"))
    assert count("split") >= 1 and count("free") == count("split")  # the node splits, freed
    assert count("bad") == 0, count("bad")
    print(f"capi: {checked} C-API loops over the Open MPI ABI bridge take the CPU path's steps bit for bit; "
          f"{count('allreduce')} MPI_Allreduce calls (all in place), {count('split')} node splits freed, no call off the ABI", flush=True)


def case_init():
    lib = iterative_solver._load()
    for name, res in (("IterativeSolver_mpi_init", C.c_int), ("IterativeSolver_mpi_finalize", C.c_int),
                      ("IterativeSolver_mpisize_global", C.c_int64), ("IterativeSolver_mpirank_global", C.c_int64)):
        getattr(lib, name).restype = res
    assert lib.IterativeSolverHbmMpiActive() == 0 and lib.IterativeSolver_mpisize_global() == 1
    assert lib.IterativeSolver_mpi_init() == 0 and count("init") == 1
    assert lib.IterativeSolverHbmMpiActive() == 1
    assert (lib.IterativeSolver_mpisize_global(), lib.IterativeSolver_mpirank_global()) == (1, 0)
    assert lib.IterativeSolver_mpicomm_global() == 0
    rng = [0, 0]
    s = iterative_solver.NonLinearEquations(10, range=rng)
    assert tuple(rng) == (0, 10)
    s.finalize()
    assert lib.IterativeSolver_mpi_finalize() == 0 and count("finalize") == 1
    assert lib.IterativeSolverHbmMpiActive() == 0 and count("bad") == 0
    print("init: MPI started and ended through the C API (Open MPI ABI)", flush=True)


if __name__ == "__main__":
    {"capi": case_capi, "init": case_init}[sys.argv[2]]()
    print(f"{sys.argv[2]} OK", flush=True)
