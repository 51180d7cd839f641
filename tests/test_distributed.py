"""The N > 1 path on CPU: index-range sharding, the select merge and the host reduction plumbing,
with world_size-2 gloo process groups (no GPU).

What the sharded product path does per op (reference util/gemm.h:157-184,
DistrArray.cpp:124-276): every rank reduces its shard, the partial results are summed over ranks
(dot, gemm_inner, sparse dot) or the per-rank top-n are all-gathered and merged identically on every
rank (select).  Here the per-shard pieces come from the oracle (the reference's loops), the
exchange goes through the product's host-communicator callbacks (subspace_hip.TorchHostComm,
what ssp_ctx_attach_host_comm calls) over gloo, and the merge is the product's ssp_select_merge;
the result must equal the unsharded oracle (select bit-exact, reductions to rounding).
The same checks also run over the stdlib-socket communicator (subspace_hip.HubComm) that the
GPU multi-rank tests use (tests/test_distributed_gpu.py).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
import subspace_hip as sh

WORLD = 2
HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_worker.py")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_torchrun(case, world=WORLD, timeout=300):
    """world ranks under torch.distributed.run, gloo process group (this process never imports
    torch: a process must hold one HIP runtime, and torch ships its own)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), WORKER, "--comm", "gloo", "--case", case]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert r.stdout.count(f"{case} OK") == world, r.stdout[-2000:]


def run_hub(case, world=WORLD, timeout=600, transport="host", env_extra=None):
    """world ranks as plain subprocesses with the stdlib-socket host communicator; transport "p2p"
    moves the reductions to the peer-memory communicator (ssp_ctx_attach_p2p, its id sent over the
    hub), the hub then only bootstraps and checks."""
    port = free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), SSP_HUB_PORT=str(port),
                   SSP_TEST_TRANSPORT=transport, **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, WORKER, "--comm", "hub", "--case", case], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rank, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {rank} failed:\n{out[-4000:]}"
        assert f"{case} OK" in out
    return outs


@pytest.mark.parametrize("n", [0, 1, 7, 8, 1000, 10**8 + 3])
@pytest.mark.parametrize("p", [1, 2, 3, 8])
def test_shard_range_is_reference_distribution(n, p):
    borders = oracle.distribution(n, p)
    for r in range(p):
        off, ln = sh.shard_range(n, p, r)
        assert (off, off + ln) == (borders[r], borders[r + 1])


def shard_select(x, nsel, p, max=False, ignore_sign=False):
    parts = []
    for r in range(p):
        off, ln = sh.shard_range(x.size, p, r)
        i, v = oracle.select(x[off:off + ln], min(nsel, ln), max=max, ignore_sign=ignore_sign)
        parts.append((i + off, v))
    return sh.select_merge(parts, nsel, max=max)


@pytest.mark.parametrize("p", [2, 3, 8])
@pytest.mark.parametrize("max,ignore_sign", [(False, False), (True, False), (False, True), (True, True)])
def test_select_merge_equals_unsharded_reference(p, max, ignore_sign):
    rng = np.random.default_rng(p * 10 + max * 2 + ignore_sign)
    # Many exact ties (small integer values), signed zeros and a ragged length.
    x = rng.integers(-4, 5, 3001).astype(float)
    x[rng.integers(0, x.size, 40)] = -0.0
    for nsel in (1, 5, 64, 700):
        gi, gv = shard_select(x, nsel, p, max, ignore_sign)
        ri, rv = oracle.select(x, nsel, max=max, ignore_sign=ignore_sign)
        np.testing.assert_array_equal(gi, ri)
        np.testing.assert_array_equal(gv, rv)


def test_select_max_dot_merge_equals_unsharded_reference():
    rng = np.random.default_rng(5)
    x, y = rng.integers(-3, 4, 999).astype(float), rng.integers(-3, 4, 999).astype(float)
    for p in (2, 5):
        parts = []
        for r in range(p):
            off, ln = sh.shard_range(x.size, p, r)
            i, v = oracle.select_max_dot(x[off:off + ln], y[off:off + ln], min(17, ln))
            parts.append((i + off, v))
        gi, gv = sh.select_merge(parts, 17, max=True)
        ri, rv = oracle.select_max_dot(x, y, 17)
        np.testing.assert_array_equal(gi, ri)
        np.testing.assert_array_equal(gv, rv)


def test_gloo_world2_sharded_reductions():
    run_torchrun("reductions")


def test_hub_world2_sharded_reductions():
    run_hub("reductions")


def test_hub_comm_collectives_world3():
    # The stdlib host communicator itself: sums identical on every rank, allgather in rank order.
    run_hub("reductions", world=3)
