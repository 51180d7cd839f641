"""The product's host code -- restated Davidson / DIIS, the HBM handlers, the reverse-communication
C API and its Python binding -- on CPU, over the host-memory emulation of the device ABI
(oracle/ssp_emul.cpp, test infrastructure), in fresh processes (tests/emul_worker.py):

* single rank: the reference's Python tests (diagonalize, non-linear equations) and the C-API
  loop taking the same iterations as the CPU reference path on the fixtures;
* world size 2 (socket host communicator, and gloo): Davidson with and without a P space, DIIS
  and the C API with shard ranges + sync, each rank holding its index range of every vector,
  against the unsharded CPU reference path (same iterations, eigenvalues within 1e-10);
* world size 8: C4's sharded Davidson and C5's sharded DIIS against the independent restatement.

The same host code over the real HIP library is tests/test_python_api_gpu.py,
tests/test_solver_gpu.py and tests/test_distributed_gpu.py.
"""
import os
import subprocess
import sys

import pytest

from test_distributed import free_port

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "emul_worker.py")


# SSP_FUSED_MIN_SIZE=0: the fused solver passes the product selects from 2^20 elements -- the one-pass
# self-orthonormalisation (ssp_axpy_gram) and the batched overlap rows (hbm_handlers.h) -- forced on
# at these sizes
ORTHO = [{}, {"SSP_FUSED_MIN_SIZE": "0"}]


@pytest.mark.parametrize("ortho", ORTHO, ids=["auto", "fused"])
def test_single_rank_api_and_loop_parity(ortho):
    r = subprocess.run([sys.executable, WORKER, "api"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, **ortho))
    assert r.returncode == 0 and "api OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("ortho", ["block", "one_pass", "two_pass"])
@pytest.mark.parametrize("arith", ["0,0", "1,1"])
def test_fused_passes_hold_the_redundancy_screen_traces(arith, ortho):
    # traces.json RS_* (N = 2^21, near-dependent R vectors: the redundancy screen removes 6 and 3 of
    # them): the product's fused numerics, which switch on from 2^20 elements, take the reference CPU
    # path's steps -- screened counts, Q sizes, working sets -- in the reference's arithmetic and in
    # a GPU-like one (8-lane sums, fma), with each self-orthonormalisation form (the block
    # form declines on most of these near-dependent sets and hands them to the sequential one)
    r = subprocess.run([sys.executable, WORKER, "rs_traces", arith], capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, SSP_ORTHO=ortho))
    assert r.returncode == 0 and "rs_traces OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_world2_sharded_solvers_socket_comm():
    port = free_port()
    procs = [subprocess.Popen([sys.executable, WORKER, "spmd"],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", SSP_HUB_PORT=str(port)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0 and "spmd OK" in out, out[-3000:]


def test_world2_sharded_solvers_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), WORKER, "spmd-gloo"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.count("OK") == 2, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("ortho", ORTHO, ids=["auto", "fused"])
def test_world8_c4_c5_sharded_against_independent_restatement(ortho):
    # the driver's 8-GPU configuration (C4: 8 roots + P 16 sharded over 8 ranks; C5: DIIS sharded) on
    # the host emulation, each rank holding its index range: the same steps as the independent
    # numpy restatement and the unsharded CPU path
    port = free_port()
    procs = [subprocess.Popen([sys.executable, WORKER, "c4"],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="8", SSP_HUB_PORT=str(port),
                                       OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", **ortho),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(8)]
    outs = [p.communicate(timeout=900)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0 and "c4 OK" in out, out[-3000:]


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_reference_distributed_array_known_answers(world):
    # testDistrArray.h / testArrayHandlerDistrSparse.cpp / testDistribution.cpp known answers on the
    # sharded ops at world sizes 1-4 (tests/distr_cases.py)
    port = free_port()
    procs = [subprocess.Popen([sys.executable, WORKER, "distr"],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), SSP_HUB_PORT=str(port),
                                       OMP_NUM_THREADS="1"),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = [p.communicate(timeout=300)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0 and "distr OK" in out, out[-3000:]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_short_solves_reproduce_the_reference_mpi_build(world):
    # tests/golden/mpi_traces.json (make_traces.py --mpi-golden): the CPU path with the dots of P MPI
    # ranks; the product's host code over the emulation on P shards, partials added in rank order,
    # must reproduce every record bit for bit (the GPU twin: test_distributed_gpu.py)
    port = free_port()
    procs = [subprocess.Popen([sys.executable, WORKER, "exact_mpi"],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), SSP_HUB_PORT=str(port),
                                       OMP_NUM_THREADS="1"),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0 and "exact_mpi OK" in out, out[-3000:]


LAUNCHER_VARS = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID", "HIP_VISIBLE_DEVICES",
                 "SSP_EMUL_DEVICES")


@pytest.mark.parametrize("env,want", [
    ({"SSP_EMUL_DEVICES": "8"}, 0),                                          # no launcher: device 0
    ({"SSP_EMUL_DEVICES": "4", "LOCAL_RANK": "5"}, 1),                       # torchrun, 5 mod 4
    ({"SSP_EMUL_DEVICES": "8", "OMPI_COMM_WORLD_LOCAL_RANK": "3"}, 3),       # Open MPI
    ({"SSP_EMUL_DEVICES": "8", "MPI_LOCALRANKID": "6"}, 6),                  # MPICH
    ({"SSP_EMUL_DEVICES": "8", "SLURM_LOCALID": "7"}, 7),                    # Slurm
    ({"SSP_EMUL_DEVICES": "8", "LOCAL_RANK": "5", "HIP_VISIBLE_DEVICES": "5"}, 0),  # one visible device
    ({"SSP_EMUL_DEVICES": "8", "LOCAL_RANK": "3", "SLURM_LOCALID": "1"}, 3),  # LOCAL_RANK first
])
def test_c_api_default_device_follows_node_local_rank(env, want):
    base = {k: v for k, v in os.environ.items() if k not in LAUNCHER_VARS}
    r = subprocess.run([sys.executable, WORKER, "devsel", str(want)], env=dict(base, **env), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "devsel OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
