"""The Open MPI ABI branch of the fcomm bridge (iterative-solver_amd/host/mpi_bridge.cpp Impl<void*>), on
CPU.  Only MPICH exists in this image, so a one-rank stand-in exporting Open MPI's symbol set
(tests/fake_ompi/fake_ompi.c, test infrastructure: ompi_mpi_comm_world, ompi_mpi_double,
ompi_mpi_op_sum, ompi_mpi_info_null, MPI_Comm_f2c / _c2f, ...) is compiled here and loaded RTLD_GLOBAL
before the product, as an Open MPI caller's process would have it (tests/ompi_worker.py).  What it
exercises: the ABI detection, handle conversion through MPI_Comm_f2c (the reference's
IterativeSolverCMPI.cpp:169) and MPI_Comm_c2f, MPI_IN_PLACE as (void*)1, the node split by
MPI_COMM_TYPE_SHARED = 0 and its MPI_Comm_free, MPI_Allreduce / _Allgather / _Bcast with Open MPI's
predefined handles, MPI_Init / _Finalize through the C API.  What it cannot: several ranks, and a real
Open MPI's reduction order.
"""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "build", "libitsolv_emul.so")),
                                reason="needs `make -C oracle`")


@pytest.fixture(scope="module")
def fake_ompi(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("fake_ompi") / "libfake_ompi.so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-o", out, os.path.join(HERE, "fake_ompi", "fake_ompi.c")],
                   check=True)
    return out


@pytest.mark.parametrize("case", ["capi", "init"])
def test_open_mpi_abi_bridge(fake_ompi, case):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("ITSOLV_HBM_COMM", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "ompi_worker.py"), fake_ompi, case],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and f"{case} OK" in r.stdout, r.stdout[-4000:] + r.stderr[-4000:]
    print(r.stdout.splitlines()[0])
