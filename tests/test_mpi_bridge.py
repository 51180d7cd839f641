"""The reference's MPI communicator argument through the C API (iterative-solver_amd/host/mpi_bridge.h),
on CPU: the product's host code over the host-memory emulation (oracle/ssp_emul.cpp) in P processes
under this container's MPICH (`mpiexec -n P`, /opt/conda MPICH 3.3.2), each process having loaded and
initialised MPI as the reference's callers do (tests/mpi_worker.py).

* MPICH's own association of MPI_Allreduce(MPI_SUM), measured (oracle_ops.c sum order 200 + P is its
  model, exact for P = 2, 3, 4, 6, 7, 8);
* the reference's C-API loops with the default communicator (IterativeSolver_mpicomm_global): the
  Initialize calls return the reference's ranges over the MPI world (IterativeSolverCMPI.cpp:79-87),
  the device follows the rank's place on its node, and every loop takes the steps of the CPU path with
  its dots summed as MPICH sums P ranks' partials, bit for bit;
* the synthetic solves of make_traces.py MPI_CASES over the "mpi" transport reproduce the committed
  MPICH records (tests/golden/mpich_traces.json) bit for bit;
* IterativeSolver_mpi_init / _mpi_finalize, and a transport the process cannot run failing on every
  rank instead of hanging.

The same loops over the HIP library on one MI355X are tests/test_mpi_bridge_gpu.py.
"""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
WORKER = os.path.join(HERE, "mpi_worker.py")
MPIEXEC = os.environ.get("MPIEXEC", "/opt/conda/bin/mpiexec")
GOLDEN = os.path.join(HERE, "golden", "mpich_traces.json")

pytestmark = pytest.mark.skipif(not (os.path.exists(MPIEXEC) and os.path.exists(os.path.join(
    ROOT, "oracle", "build", "libitsolv_emul.so"))), reason="needs MPICH's mpiexec and `make -C oracle`")


def mpirun(nproc, *args, env_extra=None, timeout=600, expect_ok=True):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    r = subprocess.run([MPIEXEC, "-n", str(nproc), sys.executable, "-u", WORKER, *args], capture_output=True,
                       text=True, timeout=timeout, env=env)
    if expect_ok:
        assert r.returncode == 0 and r.stdout.count(f"{args[0]} OK") == nproc, r.stdout[-4000:] + r.stderr[-4000:]
    return r


@pytest.mark.parametrize("nproc", [2, 3, 4, 5, 6, 8])
def test_mpich_allreduce_association(nproc):
    print(mpirun(nproc, "assoc", "emul").stdout.splitlines()[0])


@pytest.mark.parametrize("nproc", [1, 2, 3, 4, 8])
def test_capi_loops_sharded_over_mpi(nproc):
    # 3 visible devices, so that ranks 3.. wrap round: the device is the node-local rank modulo the count
    r = mpirun(nproc, "capi", "emul", env_extra={"HIP_VISIBLE_DEVICES": "0,1,2", "SSP_EMUL_DEVICES": "3"})
    print([ln for ln in r.stdout.splitlines() if ln.startswith("capi:")][0])


@pytest.mark.parametrize("nproc", [2, 3, 4, 8])
def test_synthetic_solves_match_mpich_records(nproc):
    r = mpirun(nproc, "synth", "emul", "mpi", "check", GOLDEN)
    print("\n".join(ln for ln in r.stdout.splitlines() if "bit-identical" in ln))


def test_mpi_init_and_finalize_through_the_c_api():
    mpirun(2, "init", "emul")


def test_unusable_transport_fails_every_rank():
    # the emulation has no device memory to share: p2p cannot attach, and every rank says so
    r = mpirun(2, "transport_error", "emul", "ssp_ctx_attach_p2p", env_extra={"ITSOLV_HBM_COMM": "p2p"})
    assert r.stdout.count("transport_error:") == 2
    r = mpirun(2, "transport_error", "emul", "unknown transport", env_extra={"ITSOLV_HBM_COMM": "tcp"})


def test_transport_preference_list_falls_back_on_every_rank():
    # "p2p,mpi": the peer-memory attach fails (the emulation shares no device memory), every rank learns
    # it from the agreed outcome and attaches the MPI transport in the same process; the C-API loops then
    # take the CPU path's steps with MPICH's sums, bit for bit, as under "mpi"
    r = mpirun(2, "capi", "emul", env_extra={"ITSOLV_HBM_COMM": "p2p,mpi"})
    assert "transport p2p unavailable" in r.stderr and "trying mpi" in r.stderr, r.stderr[-2000:]


def test_mpich_records_pin_the_association_model():
    # the committed records are reproduced by the restated CPU path under the association model
    # (make_mpi_traces.py re-checks this when it writes them; here without MPI)
    import json

    import numpy as np

    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(HERE, "golden")]
    import oracle
    from make_traces import MPI_CASES, mpi_options

    rec = json.load(open(GOLDEN))
    try:
        for name in ("C1_rank8", "D_1000"):
            c = MPI_CASES[name]
            fn = oracle.davidson_synthetic if c["kind"] == "davidson" else oracle.diis_synthetic
            for p in (2, 4, 8):
                oracle.set_sum_order(200 + p)
                r = fn(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **mpi_options(c))
                got = rec[name][f"mpich{p}"]
                assert r["iterations"] == got["iterations"], (name, p)
                assert np.asarray(r["trace"]["errors"]).tolist() == got["trace"]["errors"], (name, p)
    finally:
        oracle.set_sum_order(0)
