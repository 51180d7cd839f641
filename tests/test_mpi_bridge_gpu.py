"""The reference's MPI communicator argument on one MI355X (tests/test_mpi_bridge.py is the CPU form):
P processes under MPICH's `mpiexec -n P`, each with MPI loaded and initialised before the product
(tests/mpi_worker.py), all sharing the box's one device.

* the reference's C-API loops with the default communicator, over the "mpi" transport (the reductions
  MPICH's MPI_Allreduce) and the "p2p" transport (IPC-shared device inboxes): the steps of the CPU
  path with its dots summed as MPICH sums P ranks' partials, bit for bit (short vectors: the HIP
  path's reference arithmetic);
* the synthetic solves of make_traces.py MPI_CASES: bit for bit the committed MPICH records
  (tests/golden/mpich_traces.json, written by the CPU path under MPICH) -- over "mpi" at P = 2, 3, 4,
  8, and over "p2p", whose rank-order sum is MPICH's association at P = 2 and 3;
* "rccl" with two ranks on one device: refused on every rank with the reason.

Skipped when the box has no MPI runtime.
"""
import os

import pytest

from test_mpi_bridge import GOLDEN, MPIEXEC, mpirun

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no MPI runtime (mpiexec) on this machine")]


@pytest.mark.parametrize("transport,nproc", [("mpi", 2), ("mpi", 4), ("p2p", 2), ("p2p", 3)])
def test_capi_loops_sharded_over_mpi_on_hbm(transport, nproc):
    r = mpirun(nproc, "capi", "gpu", env_extra={"ITSOLV_HBM_COMM": transport, "SSP_COMM_TIMEOUT_S": "60"},
               timeout=900)
    print([ln for ln in r.stdout.splitlines() if ln.startswith("capi:")][0])


@pytest.mark.parametrize("transport,nproc", [("mpi", 2), ("mpi", 3), ("mpi", 4), ("mpi", 8), ("p2p", 2), ("p2p", 3)])
def test_synthetic_solves_match_mpich_records_on_hbm(transport, nproc):
    r = mpirun(nproc, "synth", "gpu", transport, "check", GOLDEN, env_extra={"SSP_COMM_TIMEOUT_S": "60"}, timeout=900)
    print("\n".join(ln for ln in r.stdout.splitlines() if "bit-identical" in ln))


def test_rccl_with_two_ranks_on_one_device_is_refused():
    r = mpirun(2, "transport_error", "gpu", "a device per rank", env_extra={"ITSOLV_HBM_COMM": "rccl"})
    assert r.stdout.count("transport_error:") == 2


def test_rccl_preference_list_falls_back_to_mpi_on_hbm():
    # "rccl,mpi" with two ranks on one device: RCCL is refused on every rank (agreed), every rank attaches
    # the MPI transport in the same process, and the loops take the CPU path's steps bit for bit
    r = mpirun(2, "capi", "gpu", env_extra={"ITSOLV_HBM_COMM": "rccl,mpi", "SSP_COMM_TIMEOUT_S": "60"}, timeout=900)
    assert "transport rccl unavailable" in r.stderr and "trying mpi" in r.stderr, r.stderr[-2000:]
