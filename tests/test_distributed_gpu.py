"""The sharded (N > 1) product path on a real MI355X: two ranks, each a separate process holding
its index-range shard in HBM, reductions exchanged through the host communicator
(ssp_ctx_attach_host_comm + subspace_hip.HubComm, since RCCL refuses two ranks on one device).

Everything above the transport is the code the 8-GPU RCCL runs execute: the shard ranges, the
local kernels, the reduce-then-exchange of dot / gemm_inner / sparse dots / synthetic actions,
the select all-gather + ssp_select_merge, the global-index filtering of sparse ops, and the SPMD
solver.  The bar is the unsharded reference: select bit-exact, reductions to rounding, and the
sharded Davidson / DIIS runs take the same iterations as the CPU reference path with eigenvalues
within 1e-10 (tests/dist_worker.py).
"""
import os
import subprocess
import sys
import time

import pytest

from test_distributed import WORKER, free_port, run_hub

pytestmark = pytest.mark.gpu


def test_world2_ops_on_shards():
    run_hub("gpu_ops", timeout=600)


def test_world2_davidson_and_diis_on_shards():
    run_hub("gpu_solver", timeout=900)


def test_world2_reference_distributed_array_known_answers():
    # testDistrArray.h / testArrayHandlerDistrSparse.cpp known answers on HBM shards (tests/distr_cases.py)
    run_hub("gpu_distr", timeout=300)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_traces_match_reference_path(world):
    # C4's shape (8 roots + P 16, rank-8 H) at N = 1e7, C2 and C5 (the well-posed DIIS instance, and the
    # chaotic instance's descent), sharded over 2, 3 (ragged), 4 and 8 ranks on HBM: step for step with
    # the single-rank reference CPU path's committed traces
    print(run_hub("gpu_traces", world=world, timeout=600)[0])


def test_c4_full_size_on_8_shards(monkeypatch):
    # BASELINE config C4 at full size: N = 1e8, 8 roots + P 16, rank-8 H, sharded over 8 ranks (12.5e6
    # elements, 100 MB per vector per rank, 90 GB in all) -- here 8 processes on one MI355X with the
    # host communicator in place of RCCL -- against the committed single-rank CPU-path trace of the same
    # problem at full size (traces.json C3_n1e8_rank8: 7 iterations, 48 R creations, the same steps
    # under both reordered sums) with the full bar: iterations, R/Q creations, Q-space and working-set
    # sizes after every iteration, eigenvalues within 1e-10, errors within the tolerance.
    monkeypatch.setenv("SSP_TRACES_FULL", "C4")
    print(run_hub("gpu_traces", world=8, timeout=600)[0])


def test_c5_full_size_on_8_shards(monkeypatch):
    # BASELINE config C5 at full size (DIIS, N = 1e8) over 8 ranks (8 processes on one MI355X, host
    # communicator): the committed CPU-path trace (traces.json C5_n1e8) step for step -- iterations,
    # R/Q creations, Q-space and working-set sizes -- and x = t 1 (t = 1/sqrt(N)) on every shard
    monkeypatch.setenv("SSP_TRACES_FULL", "C5")
    print(run_hub("gpu_traces", world=8, timeout=600)[0])


# ---- the peer-memory transport (ssp_ctx_attach_p2p): the multi-rank DEVICE exchange on one MI355X --
# The same cases with every reduction summed by the ranks' k_p2p_allreduce kernels through IPC-shared
# inboxes (fixed rank order, bit-identical on every rank) and the select all-gather / barriers through
# the shared host segment: the code path of a multi-rank device exchange, which RCCL cannot run with
# several ranks on one GPU.

def test_world2_ops_on_shards_p2p():
    run_hub("gpu_ops", timeout=600, transport="p2p", env_extra={"SSP_COMM_TIMEOUT_S": "60"})


def test_world2_davidson_and_diis_on_shards_p2p():
    run_hub("gpu_solver", timeout=900, transport="p2p", env_extra={"SSP_COMM_TIMEOUT_S": "60"})


def test_world2_reference_distributed_array_known_answers_p2p():
    run_hub("gpu_distr", timeout=300, transport="p2p", env_extra={"SSP_COMM_TIMEOUT_S": "60"})


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_traces_match_reference_path_p2p(world):
    print(run_hub("gpu_traces", world=world, timeout=600, transport="p2p",
                  env_extra={"SSP_COMM_TIMEOUT_S": "60"})[0])


def test_c4_full_size_on_8_shards_p2p():
    print(run_hub("gpu_traces", world=8, timeout=600, transport="p2p",
                  env_extra={"SSP_TRACES_FULL": "C4", "SSP_COMM_TIMEOUT_S": "60"})[0])


def test_c5_full_size_on_8_shards_p2p():
    print(run_hub("gpu_traces", world=8, timeout=600, transport="p2p",
                  env_extra={"SSP_TRACES_FULL": "C5", "SSP_COMM_TIMEOUT_S": "60"})[0])


# ---- rank-order sums, bit for bit (short vectors, rank-order transports) ------------------------------
# The CPU path with its dots summed as P ranks' partials added in rank order (mpi_traces.json) -- one
# valid MPI_Allreduce association; MPICH's own, through the "mpi" transport, is test_mpi_bridge_gpu.py.
@pytest.mark.parametrize("transport", ["host", "p2p"])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_short_solves_rank_order_sums(world, transport):
    # C1's shards (N = 1e4 over P ranks) and S_p8's exceed the 2048-element default on 2 ranks
    out = run_hub("gpu_exact_mpi", world=world, timeout=600, transport=transport,
                  env_extra={"SSP_COMM_TIMEOUT_S": "60", "SSP_EXACT_MAX": "16384"})[0]
    print(out)


# ---- fail fast: a lost rank ends the survivors' solves with SSP_ERR_COMM, no hang, no process left --
@pytest.mark.parametrize("transport", ["host", "p2p"])
def test_lost_rank_fails_fast(transport):
    timeout_s = 6.0
    port = free_port()
    procs = []
    t0 = time.time()
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", SSP_HUB_PORT=str(port), SSP_TEST_TRANSPORT=transport,
                   SSP_COMM_TIMEOUT_S=str(timeout_s))
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, "--comm", "hub", "--case", "gpu_peer_lost"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=100)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    print(outs[0][-2000:])
    assert procs[0].returncode == 0 and "gpu_peer_lost OK" in outs[0], outs[0][-4000:]
    if transport == "host":
        assert procs[1].returncode == 17, outs[1][-4000:]  # died mid-solve, as intended
    else:
        assert procs[1].returncode == 0 and "sees the abort" in outs[1], outs[1][-4000:]
    assert all(p.poll() is not None for p in procs)  # nothing left behind
    assert time.time() - t0 < 90
