"""The RCCL code path of libsubspace_hip.so on real hardware, on a one-GPU machine.

RCCL refuses two ranks on one device, so the multi-rank tests on one MI355X reduce through the host
communicator (test_distributed_gpu.py).  A ONE-rank RCCL communicator is legal, and with one attached
every reduction of the library goes through ncclAllReduce / ncclAllGather on the context stream
(context.hip: allreduce_dev, ssp_allgather_host) — the calls bench.py and a multi-GPU solver make
at N > 1.  Each reducing op and a whole Davidson / DIIS solve must give bit-identical results with
and without the communicator (a one-rank sum is the identity).
"""
import numpy as np
import pytest

import itsolv_hbm as ih
import subspace_hip as sh

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pair():
    if sh.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X")
    plain, comm = sh.Context(0), sh.Context(0)
    comm.attach_comm(1, 0, sh.Context.unique_id())
    yield plain, comm
    comm.close()
    plain.close()


def both(pair, fn):
    return [fn(c) for c in pair]


def test_comm_attached(pair):
    plain, comm = pair
    assert comm.lib.ssp_ctx_nranks(comm.handle) == 1 and comm.lib.ssp_ctx_rank(comm.handle) == 0


@pytest.mark.parametrize("n", [1, 1003, 1_000_003])
def test_reductions_through_rccl(pair, n):
    r = np.random.default_rng(n)
    xs = [r.uniform(-1, 1, n) for _ in range(8)]
    ys = [r.uniform(-1, 1, n) for _ in range(5)]
    a, b = both(pair, lambda c: c.dot(c.upload(xs[0]), c.upload(ys[0])))
    assert a == b
    a, b = both(pair, lambda c: c.gemm_inner([c.upload(v) for v in xs], [c.upload(v) for v in ys]))
    assert np.array_equal(a, b)
    ps = [{0: 1.0}, {n - 1: -2.0, n // 2: 0.5}]
    a, b = both(pair, lambda c: c.gemm_inner_sparse([c.upload(v) for v in xs[:3]], ps))
    assert np.array_equal(a, b)


def test_select_through_rccl_allgather(pair):
    x = np.round(np.random.default_rng(5).uniform(-30, 30, 100_003))
    (ia, va), (ib, vb) = both(pair, lambda c: c.select(c.upload(x), 16))
    assert ia.tolist() == ib.tolist() and np.array_equal(va, vb)
    (ia, va), (ib, vb) = both(pair, lambda c: c.select_max_dot(c.upload(x), c.upload(np.ones_like(x)), 5))
    assert ia.tolist() == ib.tolist() and np.array_equal(va, vb)


def test_allgather_and_barrier(pair):
    _, comm = pair
    assert comm.allgather_bytes(b"rank0-payload") == [b"rank0-payload"]
    comm.barrier()
    comm.barrier()


def test_davidson_and_diis_through_rccl(pair):
    kw = dict(nroots=4, convergence_threshold=1e-8, max_size_qspace=24, reset_D=8)
    a, b = both(pair, lambda c: ih.davidson_synthetic(c, 200_000, 0.1, 8, 7, **kw))
    assert a["iterations"] == b["iterations"]
    assert np.array_equal(a["eigenvalues"], b["eigenvalues"])
    assert np.array_equal(a["solutions"], b["solutions"])
    kw = dict(nroots=1, convergence_threshold=1e-8, max_size_qspace=6)
    a, b = both(pair, lambda c: ih.diis_synthetic(c, 100_000, 0.1, 1, 3, **kw))
    assert a["iterations"] == b["iterations"]
    assert np.array_equal(a["x"], b["x"])


def test_comm_deadline_aborts_instead_of_hanging():
    # Fail fast (context.hip wait_flag / comm_p2p.hip comm_poll): with a communicator attached, a
    # reduction whose result does not arrive within SSP_COMM_TIMEOUT_S returns SSP_ERR_COMM, the
    # communicator is aborted (ncclCommAbort) and every later exchange fails at once -- the
    # status-code form of the reference's job abort (DistrArray.cpp:16-23).  The stalled stream (a
    # bounded device spin standing in for a missing peer) ends on its own.
    import time

    c = sh.Context(0)
    c.attach_comm(1, 0, sh.Context.unique_id())
    c.set_comm_timeout(0.5)
    x = c.upload(np.ones(1000))
    assert c.dot(x, x) == 1000.0
    c.debug_stall(3000)
    t0 = time.time()
    with pytest.raises(sh.SspError) as e:
        c.dot(x, x)
    dt = time.time() - t0
    assert e.value.code == 5 and "no completion within 0.5 s" in str(e.value), e.value
    # the deadline fired at 0.5 s; ncclCommAbort then waits for the stream's work -- a stuck RCCL
    # kernel is released by the abort, this stand-in spin ends by itself at 3 s
    assert 0.4 < dt < 4.0, dt
    t0 = time.time()
    with pytest.raises(sh.SspError) as e:
        c.gemm_inner([x], [x])
    assert e.value.code == 5 and time.time() - t0 < 0.5
    with pytest.raises(sh.SspError):
        c.allgather_bytes(b"x")
    c.close()  # waits for the stall to drain


def test_p2p_deadline_aborts_instead_of_hanging():
    # The same on the peer-memory transport, whose abort only raises the shared abort word (no wait):
    # the error comes at the host deadline (timeout + min(5 s, timeout)) while the stream is still busy.
    import time

    c = sh.Context(0)
    c.attach_p2p(1, 0, sh.Context.p2p_unique_id())
    c.set_comm_timeout(0.5)
    x = c.upload(np.ones(1000))
    assert c.dot(x, x) == 1000.0
    c.debug_stall(4000)
    t0 = time.time()
    with pytest.raises(sh.SspError) as e:
        c.dot(x, x)
    dt = time.time() - t0
    assert e.value.code == 5 and "no completion within 0.5 s" in str(e.value), e.value
    assert 0.9 < dt < 2.0, dt
    with pytest.raises(sh.SspError):
        c.barrier()
    c.close()


@pytest.mark.parametrize("n", [1, 1003, 1_000_003])
def test_one_rank_p2p_transport_is_the_identity(pair, n):
    # The peer-memory transport with one rank pushes into its own inbox and sums it: every reduction
    # bit-identical to the communicator-free context (the multi-rank cases: test_distributed_gpu.py).
    plain, _ = pair
    c = sh.Context(0)
    c.attach_p2p(1, 0, sh.Context.p2p_unique_id())
    try:
        r = np.random.default_rng(n)
        xs = [r.uniform(-1, 1, n) for _ in range(8)]
        ys = [r.uniform(-1, 1, n) for _ in range(5)]
        for fn in (lambda k: k.dot(k.upload(xs[0]), k.upload(ys[0])),
                   lambda k: k.gemm_inner([k.upload(v) for v in xs], [k.upload(v) for v in ys]),
                   lambda k: k.gemm_inner_sparse([k.upload(v) for v in xs[:3]], [{0: 1.0}, {n - 1: -2.0}]),
                   lambda k: k.select(k.upload(np.round(xs[1] * 30)), min(16, n))[0].tolist()):
            assert np.array_equal(fn(plain), fn(c))
        assert c.allgather_bytes(b"abc") == [b"abc"]
        c.barrier()
    finally:
        c.close()


RCCL_ALONE = r"""
import sys, time
sys.path[:0] = [sys.argv[1]]
import subspace_hip as sh
c = sh.Context(0)
c.set_comm_timeout(float(sys.argv[2]))
t0 = time.time()
try:
    c.attach_comm(2, 0, sh.Context.unique_id())  # rank 1 never joins
    print("ATTACHED")
except sh.SspError as e:
    print(f"FAILED {e.code} {time.time() - t0:.2f} {e}")
c.close()
"""


def test_rccl_join_without_the_other_rank_fails_within_the_deadline():
    # The driver's N > 1 bench joins an RCCL communicator; a rank that never arrives must end the join
    # of the others with SSP_ERR_COMM_ABANDONED after SSP_COMM_TIMEOUT_S instead of waiting for ever.
    # The blocking ncclCommInitRank runs on a helper thread that the caller stops waiting for at the
    # deadline (the thread stays inside RCCL's bootstrap, so the process must end: no later attach,
    # INTEGRATION.md §5) -- and the process still exits and leaves nothing behind.
    import os
    import subprocess
    import sys
    import time

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "iterative-solver_amd")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", RCCL_ALONE, pkg, "8"], capture_output=True, text=True, timeout=90)
    wall = time.time() - t0
    print(r.stdout[-1500:], r.stderr[-1500:])
    assert r.returncode == 0 and "FAILED 8" in r.stdout, r.stdout + r.stderr
    took = float(r.stdout.split("FAILED 8 ")[1].split()[0])
    assert 7.5 < took < 20, took
    assert "did not form within 8 s" in r.stdout
    assert wall < 80
