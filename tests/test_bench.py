"""bench.py: the driver's contract (one JSON line from rank 0 with the required keys) and its helpers.

CPU: shard borders, algorithmic bytes per step, the PMC-summary lookup, the CPU baseline leg.
GPU: a short N = 1 run, and N = 2 launched exactly as the driver launches it
(`python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 ...`)
with `--comm host`, two ranks on the box's one device (RCCL refuses duplicate GPUs; the RCCL calls
themselves are covered by test_rccl_gpu.py).
"""
import json
import os
import subprocess
import sys

import pytest

import oracle
from test_distributed import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


@pytest.mark.parametrize("n,p", [(10**8, 1), (10**8, 8), (10**8 + 3, 8), (7, 3)])
def test_distribution_is_reference(n, p):
    assert bench.distribution(n, p) == oracle.distribution(n, p).tolist()


def test_step_bytes():
    # 2 x gemm_inner 8N(m+k) + 2 m fills 8N + 2 x gemm_outer 8N(k+2m) + m axpy 24N + m dot 8N
    n, m, k = 10**8, 8, 48
    assert bench.step_bytes(n, m, k) == 8 * n * (2 * (m + k) + 2 * m + 2 * (k + 2 * m) + 3 * m + m)
    assert bench.step_bytes(n, m, k) == 230.4e9


def test_pmc_traffic_lookup():
    path = os.path.join(ROOT, "profiles", "r1", "pmc_traffic_n1e8.json")
    t, src = bench.pmc_traffic(path, "gemm_outer", 10**8, 8, 48, 1)
    assert t is not None and src.startswith("profiles/r1/pmc_traffic_n1e8.json:k_gemm_outer")
    assert abs(t - 8 * 10**8 * (48 + 16)) / t < 0.02  # algorithmic bytes: no re-reads
    assert bench.pmc_traffic(path, "gemm_outer", 10**8, 8, 48, 2) == (None, None)  # other workload
    assert bench.pmc_traffic("/nonexistent.json", "dot", 1, 1, 1, 1) == (None, None)


def test_pmc_traffic_lookup_r2_names_the_rmw_instance():
    # r2's summary holds both gemm_outer instances; the roofline kernel is the read-modify-write one
    path = os.path.join(ROOT, "profiles", "r2", "pmc_traffic_n1e8.json")
    t, src = bench.pmc_traffic(path, "gemm_outer", 10**8, 8, 48, 1)
    assert src.endswith("k_gemm_outer<8, false, false>") and abs(t - 8 * 10**8 * (48 + 16)) / t < 0.02
    t, src = bench.pmc_traffic(path, "gemm_outer_set", 10**8, 8, 48, 1)
    assert src.endswith("k_gemm_outer<8, false, true>") and abs(t - 8 * 10**8 * (48 + 8)) / t < 0.02


def test_pmc_traffic_lookup_r6_default():
    # the file bench.py reports as roofline.traffic by default (round-6 final tree): the RMW gemm_outer
    # moves its algorithmic bytes, read 48 + 8 vectors, write 8
    path = os.path.join(ROOT, "profiles", "r6", "pmc_traffic_n1e8_r6.json")
    t, src = bench.pmc_traffic(path, "gemm_outer", 10**8, 8, 48, 1)
    assert src == "profiles/r6/pmc_traffic_n1e8_r6.json:k_gemm_outer<8, false, false, false>"
    assert abs(t - 8 * 10**8 * (48 + 16)) / t < 1e-4


def test_mfma_util_lookup():
    path = os.path.join(ROOT, "profiles", "r1", "mfma_util_n1e8.json")
    util, src = bench.mfma_util(path)
    assert 0 < util < 100 and src.startswith("profiles/r1/mfma_util_n1e8.json:k_gemm_inner<2, 12")
    d = json.load(open(path))
    k = next(v for n, v in d["bench_step"].items() if n.startswith("k_gemm_inner<2, 12"))
    assert k["mfma_f64_flops_per_dispatch"] == 2 * 8 * 48 * 10**8  # MOPS x 512 = algorithmic flops
    assert bench.mfma_util("/nonexistent.json") == (None, None)


def test_cpu_baseline_leg():
    # in a thread, as bench.py runs it: the leg pins its own thread to one core (never the caller's)
    import threading

    box = {}
    th = threading.Thread(target=lambda: box.update(cb=bench.cpu_baseline_core(2, 3, 0.05, n=200_000),
                                                    solve=bench.cpu_solve_core(n=20_000)))
    before = os.sched_getaffinity(0)
    th.start()
    th.join()
    assert os.sched_getaffinity(0) == before
    cb, cs = box["cb"], box["solve"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["unit"] == "GB/s" and cb["value"] > 0
    assert "pinned: cpu" in cb["sample"] and cs["cores"] == 1 and cs["converged"] and cs["iterations"] > 0
    bench.cpu_baseline_extras(cb, 2, 3, 0.05)
    hp = cb["host_parallel"]
    assert hp["kind"] == "host-parallel" and hp["cores"] >= 1 and hp["value"] > 0


def parse(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    d = json.loads(lines[0])
    assert KEYS <= set(d), set(KEYS) - set(d)
    assert d["value"] > 0 and d["unit"] == "GB/s" and d["dtype"] == "f64" and d["higher_is_better"] is True
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] < 1.0
    return d


@pytest.mark.gpu
def test_bench_single_gpu():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--n-global", "4e6",
           "--cpu-seconds", "0.5", "--cpu-n", "1e6", "--cpu-solve-n", "1e5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["cpu_baseline"]["value"] > 0
    assert d["config"]["n_global"] == 4_000_000
    # the roofline ledger is the timed region: every op of the 3 steps carries its event pair
    assert d["ledger"].startswith("HIP events around every op") and d["ops"]["gemm_outer"]["calls_per_step"] == 2
    assert d["sustained"]["steps"] >= 5 and d["sustained"]["GBs"] > 0
    s = d["in_solver_cpu"]
    assert s["cpu"]["converged"] and s["same_iterations"] and s["speedup"] > 0
    c4 = d["in_solver_c4_shard"]  # one rank's share of C4 (N / 8)
    assert c4["n_global"] == 500_000 and c4["converged"] and c4["config"].startswith("C4, one rank's share")


@pytest.mark.gpu
def test_bench_two_ranks_host_hub():
    env = dict(os.environ)
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--n-global", "4000001", "--comm", "host"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 2 and d["cpu_baseline"] is None
    assert d["config"]["n_local_rank0"] == 2_000_001  # spread-remainder: rank 0 takes the extra element


@pytest.mark.gpu
def test_bench_two_ranks_rccl_refused_falls_back_to_the_host_hub():
    # the driver's launch with the default --comm rccl, two ranks on the box's one device: RCCL's join
    # fails (a duplicate device), every rank agrees through the file rendezvous and attaches the host
    # hub in the same process, and rank 0's line names the transport that produced the value
    env = dict(os.environ, SSP_COMM_TIMEOUT_S="60")
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--n-global", "4000001", "--no-in-solver"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 2 and d["comm"] == "host" and d["comm_fallback"]["from"] == "rccl"
    assert "host-hub" in d["config"]["parallelism"]


@pytest.mark.gpu
@pytest.mark.parametrize("comm", ["p2p", "auto"])
def test_bench_two_ranks_peer_memory(comm):
    # the driver's launch with the peer-memory transport (two ranks on the one device): the attach
    # self-test passes, the reductions run through k_p2p_allreduce, one JSON line
    env = dict(os.environ)
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--n-global", "4000001", "--comm", comm]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 2 and "peer-memory" in d["config"]["parallelism"]
    assert d["in_solver"]["converged"] and d["in_solver"].get("same_steps_as_cpu_path") is not False


def test_bench_eight_ranks_emulated():
    """The driver's 8-GPU launch rehearsed on CPU: 8 ranks under torch.distributed.run over the host
    emulation of the device ABI (--comm host): shard sizes, barriers, max-over-ranks time, ledger and
    one JSON line from rank 0."""
    env = dict(os.environ)
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    n = 8 * 12_500 + 5
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "bench_emul.py"), "bench",
           "--gpus", "8", "--steps", "2", "--warmup", "1", "--ledger-steps", "1", "--n-global", str(n),
           "--comm", "host"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 8 and d["cpu_baseline"] is None and d["scaling"] == "strong"
    assert d["config"]["n_local_rank0"] == bench.distribution(n, 8)[1] == 12_501
    assert d["config"]["bytes_per_step"] == bench.step_bytes(n, 8, 48)
    assert set(d["ops"]) == {"gemm_inner", "gemm_outer", "fill", "axpy", "dot"}
    # the product's own form of the step, and the sharded whole solve (config C4's shape)
    assert d["product_step"]["bytes_per_step"] == bench.product_step_bytes(n, 8, 48)
    assert set(d["product_step"]["ops"]) == {"gemm_inner", "gemm_outer_set", "axpy_pairs_norm"}
    s = d["in_solver"]
    assert s["converged"] and s["iterations"] > 0 and s["n_global"] == n and s["reductions_per_iteration"] > 0


def test_rccl_id_rendezvous_eight_ranks():
    """bench.rendezvous_uid: rank 0's RCCL unique id reaches all 8 local ranks (siblings of one
    launcher process, keyed by MASTER_ADDR/PORT and the parent pid)."""
    port = str(free_port())
    procs = []
    for r in range(8):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="8", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "bench_emul.py"), "uid"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                      cwd=ROOT))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    want = bytes(range(7, 7 + 128)).hex()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, out[-2000:]
        assert f"uid {r} {want}" in out, out[-2000:]


def test_bench_eight_ranks_rccl_join_failure_falls_back_to_the_host_hub():
    """The driver's 8-GPU launch with the default --comm rccl when one rank's RCCL join fails: every
    rank learns it through the launcher's file rendezvous and attaches the host hub in the same
    process, and rank 0 prints one JSON line naming the transport that produced the value.  Over the
    host emulation, whose RCCL join "succeeds" on the other ranks (SSP_EMUL_RCCL_JOIN=1); rank 3's
    attach is made to fail (SSP_BENCH_FAIL_RCCL_RANK=3)."""
    env = dict(os.environ, SSP_EMUL_RCCL_JOIN="1", SSP_BENCH_FAIL_RCCL_RANK="3", SSP_COMM_TIMEOUT_S="60")
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    n = 8 * 12_500 + 5
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "bench_emul.py"), "bench",
           "--gpus", "8", "--steps", "2", "--warmup", "1", "--ledger-steps", "1", "--n-global", str(n),
           "--no-in-solver"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = parse(r.stdout)
    assert d["n_gpus"] == 8 and d["comm"] == "host" and "host-hub" in d["config"]["parallelism"]
    assert d["comm_fallback"]["from"] == "rccl" and d["comm_fallback"]["failed_ranks"] == [3]
    assert r.stderr.count("every rank falls back to the host hub") == 8
