#!/usr/bin/env python3
"""bench.py — subspace-update GB/s (gemm_inner + gemm_outer/axpy + dot) at N = 1e8, 8 roots.

One "step" is the handler-operation sequence of one Davidson subspace update at steady state
(reference call stack SURVEY.md §3.1; every op is a libsubspace_hip.so C-ABI call on HBM-resident
shards):
  S_RQ = gemm_inner(R params (m), Q params (k))        XSpace.h:43      8N(m+k) B
  H_RQ = gemm_inner(R params (m), Q actions (k))       XSpace.h:47      8N(m+k) B
  construct_solution(params):  fill(0) x m, gemm_outer(k -> m)        IterativeSolverTemplate.h:46,63
  construct_solution(actions): fill(0) x m, gemm_outer(k -> m)        8N m + 8N(k+2m) B each
  residual r_i -= lambda_i x_i: axpy x m               LinearEigensystemDavidson.h:191   24N B
  errors |r_i|: dot(r_i, r_i) x m                      IterativeSolverTemplate.h:99      8N B
Global N is fixed and sharded by index range over the ranks (strong scaling, config C4); each
rank runs the identical SPMD sequence and the reductions are RCCL allreduces.

value = algorithmic bytes of all ranks per step x steps / (max over ranks of the timed wall time).

Beside the headline the JSON line carries (none of them inside the timed region):
  product_step  the same update as the product's solver runs it: construct_solution as ONE
                write-only pass per space (ssp_gemm_outer_set, IterativeSolverTemplate.h:33-65 fused,
                8N(k + m) B) and the residuals with their norms as one pass (construct_residual +
                update_errors, ssp_axpy_pairs_norm: 24N B per root, one reduction);
  in_solver     whole LinearEigensystemDavidson solves (C3 at N = 1: 8 roots + P 16, rank-8 problem,
                N = 1e8; at N > 1 the same solve sharded, BASELINE config C4): iterations, wall time,
                kernel time and algorithmic bytes from the HIP-event ledger, reductions per iteration;
  in_solver_diis  the same for NonLinearEquationsDIIS on BASELINE config C5's problem (N = 1e8, sharded
                at N > 1);
  headline_step_at_n_div_10   the headline step at N / 10 (C2's length at N = 1e8);
  startup       context creation and the first (cold) solve against the warm one;
  cpu_baseline.dram_resident  one call each of the reference loops on DRAM-resident operands.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "iterative-solver_amd"))

import numpy as np  # noqa: E402

import subspace_hip as sh  # noqa: E402

METRIC = "subspace-update GB/s (gemm_inner+axpy) at N=1e8, 8 roots; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
MFMA_F64_PEAK_TFLOPS = 78.6  # MI355X dense f64 matrix peak
SEED = 20251015


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def distribution(n, chunks):
    """Shard borders from ssp_shard_range (make_distribution_spread_remainder, reference
    util/Distribution.h:99-109)."""
    return [sh.shard_range(n, chunks, r)[0] for r in range(chunks)] + [n]


def step_bytes(n, m, k):
    return (2 * 8 * n * (m + k)      # two gemm_inner
            + 2 * m * 8 * n          # fills in construct_solution
            + 2 * 8 * n * (k + 2 * m)  # two gemm_outer
            + m * 24 * n             # residual axpy
            + m * 8 * n)             # norm dots (x == y: one vector read)


def product_step_bytes(n, m, k):
    return (2 * 8 * n * (m + k)      # two gemm_inner
            + 2 * 8 * n * (k + m)    # two write-only construct_solution passes (gemm_outer_set)
            + m * 24 * n)            # residuals and their norms in one pass (ssp_axpy_pairs_norm)


class Workload:
    def __init__(self, ctx, n_local, offset, m, k):
        self.ctx, self.m, self.k = ctx, m, k
        self.rp = [ctx.alloc(n_local) for _ in range(m)]
        self.ra = [ctx.alloc(n_local) for _ in range(m)]
        self.qp = [ctx.alloc(n_local) for _ in range(k)]
        self.qa = [ctx.alloc(n_local) for _ in range(k)]
        for vid, v in enumerate(self.rp + self.ra + self.qp + self.qa):
            ctx.fill_random(v, SEED, vid, offset)
        rng = np.random.default_rng(SEED)
        self.coef = rng.uniform(-0.1, 0.1, (k, m))
        self.lam = rng.uniform(0.5, 2.0, m)
        ctx.synchronize()

    def step(self):
        c = self.ctx
        c.gemm_inner(self.rp, self.qp)
        c.gemm_inner(self.rp, self.qa)
        for v in self.rp:
            c.fill(0.0, v)
        c.gemm_outer(self.coef, self.qp, self.rp)
        for v in self.ra:
            c.fill(0.0, v)
        c.gemm_outer(self.coef, self.qa, self.ra)
        for i in range(self.m):
            c.axpy(-self.lam[i], self.rp[i], self.ra[i])
        err = 0.0
        for i in range(self.m):
            err = max(err, c.dot(self.ra[i], self.ra[i]))
        return err

    def free(self):
        for v in self.rp + self.ra + self.qp + self.qa:
            v.free()
        self.ctx.synchronize()

    def product_step(self):
        """The same update as the product's solver issues it (see the module docstring)."""
        c = self.ctx
        c.gemm_inner(self.rp, self.qp)
        c.gemm_inner(self.rp, self.qa)
        c.gemm_outer_set(self.coef, self.qp, self.rp)
        c.gemm_outer_set(self.coef, self.qa, self.ra)
        nrm2 = c.axpy_pairs_norm(-self.lam, self.rp, self.ra)
        return float(np.max(nrm2))


def op_kernels(op, m):
    """rocprofv3 kernel-name prefixes of `op`'s main kernel for m destinations / rows (the template
    instance the launcher picks, unscaled operands; older summaries predate the SET and SC parameters)."""
    mt = next(v for v in (1, 2, 4, 8, 16) if m <= v or v == 16)
    return {"gemm_inner": ("k_gemm_inner<",),
            "gemm_outer": (f"k_gemm_outer<{mt}, false, false, false>", f"k_gemm_outer<{mt}, false, false>",
                           f"k_gemm_outer<{mt}, false>"),
            "gemm_outer_set": (f"k_gemm_outer<{mt}, false, true, false>", f"k_gemm_outer<{mt}, false, true>"),
            "axpy": ("k_axpy",), "fill": ("k_fill(",),
            "dot": ("k_dot_partial",)}.get(op, ())


def pmc_traffic(path, op, n_global, m, k, world):
    """HBM bytes per launch of `op`'s main kernel from a committed rocprofv3 --pmc summary
    (tools/pmc_summary.py: FETCH_SIZE x 2 + WRITE_SIZE, gfx950 corrections) of THIS workload."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    w = d.get("workload") or {}
    if (w.get("n_global"), w.get("roots"), w.get("qspace"), w.get("n_gpus")) != (n_global, m, k, world):
        return None, None
    for prefix in op_kernels(op, m):
        for name, v in d["kernels"].items():
            if name == prefix.rstrip("(<") or name.startswith(prefix):
                return v["hbm_bytes_per_dispatch"], os.path.relpath(path, ROOT) + ":" + name
    return None, None


def mfma_util(path, kernel_prefix="k_gemm_inner<2, 12"):
    """MFMA utilisation of gemm_inner 8x48 from the committed rocprofv3 --pmc MfmaUtil summary."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    for name, v in d.get("bench_step", {}).items():
        if name.startswith(kernel_prefix):
            return v["mfma_util_pct"], os.path.relpath(path, ROOT) + ":" + name
    return None, None


def rendezvous_uid(rank, world, timeout=300.0, kind="rccl"):
    """A communicator id (RCCL unique id, or kind "p2p": the peer-memory communicator's name) from
    rank 0 to every rank of this node through a file keyed by the launcher (MASTER_ADDR/PORT and the
    parent pid all local ranks share).  No torch in this process: it would bring a second HIP runtime
    next to libsubspace_hip.so's."""
    tag = "{}_{}_{}".format(os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                            os.getppid())
    path = os.path.join(tempfile.gettempdir(), f"ssp_bench_{kind}_uid_{tag}")
    if rank == 0:
        uid = sh.Context.p2p_unique_id() if kind == "p2p" else sh.Context.unique_id()
        with open(path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(path + ".tmp", path)
        return uid, path
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no RCCL id at {path}")
        time.sleep(0.05)
    with open(path, "rb") as f:
        return f.read(), None


def gpu_c2_solve(ctx, world, n=None):
    """The same C2 solve on the GPU(s) (sharded at N > 1), for in_solver_cpu's like-for-like ratio."""
    import itsolv_hbm as ih

    kw = dict(C2_SOLVE, **({"n": int(n)} if n else {}))
    n, rho, rank, seed = kw.pop("n"), kw.pop("rho"), kw.pop("rank"), kw.pop("seed")
    ih.davidson_synthetic(ctx, n, rho, rank, seed, n_local=0, solutions=False, **kw)  # warm
    ctx.synchronize()
    t0 = time.perf_counter()
    r = ih.davidson_synthetic(ctx, n, rho, rank, seed, n_local=0, solutions=False, **kw)
    ctx.synchronize()
    wall = time.perf_counter() - t0
    # the same solve once more under the HIP-event ledger: kernel time, rate and idle, as the other
    # in-solver blocks report them
    ctx.ledger_reset()
    ctx.ledger_enable(True)
    ih.davidson_synthetic(ctx, n, rho, rank, seed, n_local=0, solutions=False, **kw)
    ctx.synchronize()
    ctx.ledger_enable(False)
    led = ctx.ledger()
    ms = sum(v["ms"] for v in led.values())
    nb = sum(v["bytes"] for v in led.values())
    top = sorted(led.items(), key=lambda kv: -kv[1]["ms"])[:4]
    return {"wall_s": round(wall, 4), "iterations": r["iterations"],
            "r_creations": r["r_creations"], "eigenvalues": [round(float(e), 12) for e in r["eigenvalues"][:4]],
            "kernel_ms_rank0": round(ms, 3), "algorithmic_GB_rank0": round(nb / 1e9, 2),
            "kernel_GBs_rank0": round(nb / (ms / 1e3) / 1e9, 1) if ms else None,
            "idle_frac_of_wall": round((wall - ms / 1e3) / wall, 4),
            "top_ops": {op: {"calls": v["calls"], "ms": round(v["ms"], 2),
                             "GBs": round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1) if v["ms"] else None}
                        for op, v in top}}


def pin_this_thread():
    """Pins the calling thread (only it: Linux sched_setaffinity of tid 0) to one host core -- the
    last one this process may use, away from the thread that drives the GPU -- and returns it."""
    try:
        core = max(os.sched_getaffinity(0))
        os.sched_setaffinity(0, {core})
        return core
    except (AttributeError, OSError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_N = 10_000_000  # N in {1e7, 1e8}; 112 vectors of 80 MB, far beyond the host caches


def cpu_baseline_core(m, k, seconds, n=CPU_N):
    """The 1-core leg of cpu_baseline: the reference loops (oracle_ops.c: sequential dot / axpy,
    pairwise gemm_inner_default / gemm_outer_default, ArrayHandlerIterable.h:65-82, gemm.h:257-279)
    running the headline step's op sequence on DRAM-resident operands at N = 1e7, on one pinned core.
    Whole steps only: at least one, until `seconds` have passed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    core = pin_this_thread()
    runner = oracle.CpuUpdateStep(n, m, k, SEED)
    t0 = time.perf_counter()
    steps = 0
    while True:
        runner.step()
        steps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    del runner
    return {
        "value": step_bytes(n, m, k) * steps / dt / 1e9,
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{steps} step(s) of the headline op sequence at N={n:.0e} (m={m}, k={k}; {2 * (m + k)} vectors, "
                  f"{16 * (m + k) * n / 1e9:.1f} GB, DRAM-resident) on 1 core (pinned: cpu {core}) of {cpu_model()} (nproc={os.cpu_count()}), "
                  f"{dt:.1f} s, oracle/oracle_ops.c (reference loops: sequential dot/axpy, pairwise gemm)",
    }


# BASELINE.md §3 "In-solver": a whole LinearEigensystemDavidson on the rank-one H = diag(1 + i) + rho 1 1^T
# (rho = 0.1, test_rayleigh_quotient.cpp:37-42) at BASELINE config C2's size (N = 1e7, 4 roots); the
# committed CPU-path trace of the same solve is traces.json C2_rank1
C2_SOLVE = dict(n=10_000_000, rho=0.1, rank=1, seed=1, nroots=4, max_p=0, max_size_qspace=24, reset_D=8,
                convergence_threshold=1e-8)


def cpu_solve_core(n=None):
    """The in-solver CPU baseline: the oracle's C2 solve (the reference's Davidson over its CPU
    handlers, the same restated solver headers) on one pinned core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    core = pin_this_thread()
    kw = dict(C2_SOLVE, **({"n": int(n)} if n else {}))
    n, rho, rank, seed = kw.pop("n"), kw.pop("rho"), kw.pop("rank"), kw.pop("seed")
    t0 = time.perf_counter()
    r = oracle.davidson_synthetic(n, rho, rank, seed, solutions=False, **kw)
    dt = time.perf_counter() - t0
    return {"wall_s": round(dt, 3), "iterations": r["iterations"], "r_creations": r["r_creations"],
            "converged": bool(r["converged"]), "cores": 1, "pinned_core": core, "kind": "port",
            "eigenvalues": [round(float(e), 12) for e in r["eigenvalues"][:4]]}


def cpu_baseline_extras(cb, m, k, seconds):
    """host-parallel (every host thread) and the DRAM-resident single calls, run with the GPU idle."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    cb["host_parallel"] = host_parallel(m, k, max(1.0, seconds / 3))
    dram = {op: {kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in d.items()}
            for op, d in oracle.dram_resident_sample(SEED).items()}
    cb["dram_resident"] = dict(dram, note="one call each on 1 core, operands far beyond the host caches")


def host_parallel(m, k, seconds):
    """SURVEY.md §8d's second CPU figure: the same op sequence with OpenMP on all the host threads
    this process may use and cache-blocked gemm (oracle/host_parallel.c) -- "host-parallel", not
    the reference."""
    import oracle  # test infrastructure: the CPU baseline leg only

    n = 4_000_000
    runner = oracle.HostParallelStep(n, m, k, SEED)
    runner.step()
    t0 = time.perf_counter()
    steps = 0
    while True:
        runner.step()
        steps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": step_bytes(n, m, k) * steps / dt / 1e9, "unit": "GB/s", "cores": runner.threads,
            "kind": "host-parallel",
            "sample": f"{steps} step(s) at N=4e6 (m={m}, k={k}), OpenMP x{runner.threads}, {dt:.1f} s, "
                      "oracle/host_parallel.c (blocked gemm, not the reference's pairwise loops)"}


C3 = dict(rho=0.1, rank=8, seed=1, nroots=8, max_p=16, max_size_qspace=48, reset_D=8, convergence_threshold=1e-8)
# BASELINE config C5 (NonLinearEquationsDIIS, N = 1e8): the well-posed instance of tests/golden/traces.json
# C5_n1e7 / C5_n1e8 (itsolv_hbm.c5_spec: r = H (x - t 1), t = 1/sqrt(N), x from e_0, the reference test's
# 1 1^T + diag form of test_NonLinearEquations.cpp:25-49 with the coupling scaled by 1/N and a bounded
# diagonal)
C5_OPTIONS = dict(max_size_qspace=6, convergence_threshold=1e-8)
TRACES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "traces.json")


def cpu_trace(kind, n_global):
    """The committed reference-CPU-path trace of this solve, if there is one (parity evidence only)."""
    name = {("diis", 10**7): "C5_n1e7", ("diis", 10**8): "C5_n1e8",
            ("davidson", 10**8): "C3_n1e8_rank8", ("davidson", 10**7): "C3_n1e7_rank8"}.get((kind, int(n_global)))
    try:
        with open(TRACES) as f:
            t = json.load(f)
    except OSError:
        return None, None
    ref = t.get(name) if name else None
    if ref and kind == "davidson" and ref["options"].get("max_size_qspace") != C3["max_size_qspace"]:
        return None, None
    return name, ref
REDUCING_OPS = ("dot", "gemm_inner", "axpy_inner", "scal_inner", "axpy_norm", "axpy_gram", "axpy_pairs_norm", "select", "gemm_inner_sparse")


def in_solver(ctx, n_global, world, barrier, repeat=5, kind="davidson"):
    """Whole solves: Davidson with C3's options (sharded over the ranks = C4 at N > 1) or, kind =
    "diis", NonLinearEquationsDIIS with C5's.  The first (cold) solve and the warm ones after it run
    without the ledger -- their wall times carry no HIP-event records -- and the last one with it, for
    the kernel time and bytes.  Returns the median warm wall time (repeat - 2 warm solves: one solve's
    wall moves by a few percent with the host's jitter), the cold one, and the ledgered solve's numbers."""
    import itsolv_hbm as ih

    def allmax(x):
        if world == 1:
            return x
        return max(struct.unpack("<d", b)[0] for b in ctx.allgather_bytes(struct.pack("<d", x)))

    walls, has = [], []
    for rep in range(repeat):
        ctx.ledger_reset()
        ctx.ledger_enable(rep == repeat - 1)  # the last solve: the ledger
        barrier()
        t0 = time.perf_counter()
        if kind == "diis":
            r = ih.diis_synthetic(ctx, n_global, n_local=0, solutions=False, **ih.c5_spec(n_global), **C5_OPTIONS)
        else:
            r = ih.davidson_synthetic(ctx, n_global, n_local=0, **C3)
        ctx.synchronize()
        walls.append(allmax(time.perf_counter() - t0))
        ctx.ledger_enable(False)
        if 0 < rep < repeat - 1:
            has.append(r["host_algebra"])  # the warm solves' host subspace algebra
    warm = float(np.median(walls[1:-1]))
    ha = sorted(has, key=lambda h: h["seconds"])[len(has) // 2]
    led = ctx.ledger()
    ms = sum(v["ms"] for v in led.values())
    nb = sum(v["bytes"] for v in led.values())
    red = sum(v["calls"] for op, v in led.items() if op.split("(")[0] in REDUCING_OPS or op.startswith("select"))
    it = max(1, r["iterations"])
    top = sorted(led.items(), key=lambda kv: -kv[1]["ms"])[:6]
    tname, ref = cpu_trace(kind, n_global)
    parity = {}
    if ref is not None:
        same = (r["iterations"] == ref["iterations"] and r["r_creations"] == ref["r_creations"]
                and list(r["trace"]["nq"]) == ref["trace"]["nq"] and list(r["trace"]["nwork"]) == ref["trace"]["nwork"])
        parity = {"cpu_path_trace": f"tests/golden/traces.json:{tname}", "cpu_path_iterations": ref["iterations"],
                  "same_steps_as_cpu_path": bool(same)}
    if kind == "diis":
        c5 = ih.c5_spec(n_global)
        config = ("NonLinearEquationsDIIS C5: r = H (x - t 1), t = 1/sqrt(N), H = diag(1 + 2 frac(i phi)) + (1/N) 1 1^T, "
                  f"x from e_0, approximate preconditioner diagonal (alpha {c5['alpha']}), max_size_qspace 6, "
                  "threshold 1e-8"
                  + (f", sharded over {world} ranks" if world > 1 else ""))
    else:
        config = ("LinearEigensystemDavidson " + ("C3" if world == 1 else "C4") + ": 8 roots + P 16, rank-8 "
                  "H = diag(1+i) + 0.1 sum u u^T, max_size_qspace 48, reset_D 8, threshold 1e-8")
    return {
        "config": config,
        "n_global": n_global,
        "converged": bool(r["converged"]),
        "iterations": r["iterations"],
        "r_creations": r["r_creations"],
        "wall_s": round(warm, 4),
        "wall_s_warm_all": [round(w, 4) for w in walls[1:-1]],
        "wall_s_cold": round(walls[0], 4),
        "wall_s_ledger_on": round(walls[-1], 4),
        "idle_frac_of_wall": round((warm - ms / 1e3) / warm, 4),
        # of that idle: the host's subspace algebra (eigenproblem / svd_system / solve_DIIS, dense.h)
        "host_algebra_ms_rank0": round(1e3 * ha["seconds"], 3),
        "host_algebra_calls": ha["calls"],
        "host_algebra_max_dim": ha["max_dim"],
        "kernel_ms_rank0": round(ms, 3),
        "algorithmic_GB_rank0": round(nb / 1e9, 2),
        "kernel_GBs_rank0": round(nb / (ms / 1e3) / 1e9, 1) if ms else None,
        "wall_GBs_all_ranks": round(world * nb / warm / 1e9, 1),
        "reductions_per_iteration": round(red / it, 1),
        "top_ops": {op: {"calls": v["calls"], "ms": round(v["ms"], 2),
                         "GBs": round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1) if v["ms"] else None}
                    for op, v in top},
        "eigenvalues": [round(float(e), 12) for e in r["eigenvalues"][:8]] if kind != "diis" else None,
        "final_error": float(r["errors"][0]) if kind == "diis" else None,
        **parity,
    }


def setup_context(args, world, rank, local_rank):
    """This rank's context on its device, with the rank transport attached at N > 1.  Every wait on
    the other ranks -- RCCL's join included (a helper thread under the deadline; csrc/context.hip) -- is
    bounded by SSP_COMM_TIMEOUT_S (120 s here unless set).  A failed RCCL join on any rank makes every
    rank fall back to the host hub in the same process; any other setup failure ends the run with an
    error record (main) instead of a hang."""
    ctx = sh.Context(local_rank % max(1, sh.device_count()))
    if world > 1:
        ctx.set_comm_timeout(float(os.environ.get("SSP_COMM_TIMEOUT_S", "120")))
    if args.comm == "host":
        if world > 1:
            port = int(os.environ.get("MASTER_PORT", "29500")) + 1
            ctx.attach_host_comm(sh.HubComm(rank, world, os.environ.get("MASTER_ADDR", "127.0.0.1"), port))
        return ctx
    # one GPU per rank; a launcher that narrows HIP_VISIBLE_DEVICES per rank leaves one visible
    transport = "rccl"
    if world > 1 and args.comm in ("p2p", "auto"):
        uid, uid_path = rendezvous_uid(rank, world, kind="p2p")
        try:
            ctx.attach_p2p(world, rank, uid)  # collective, self-tested, the verdict agreed by all ranks
            transport = "p2p"
        except sh.SspError as e:
            if args.comm == "p2p":
                raise
            log(f"rank {rank}: peer-memory transport unavailable ({e}); using RCCL")
        if uid_path:  # attach returned on rank 0: every rank has read the id
            os.remove(uid_path)
    if world > 1 and transport == "rccl":
        err, uid_path = None, None
        try:
            uid, uid_path = rendezvous_uid(rank, world, timeout=float(os.environ.get("SSP_COMM_TIMEOUT_S", "120")))
            if os.environ.get("SSP_BENCH_FAIL_RCCL_RANK") == str(rank):  # rehearsal of a failed join
                raise sh.SspError(5, "injected RCCL attach failure (SSP_BENCH_FAIL_RCCL_RANK)")
            ctx.attach_comm(world, rank, uid)  # collective: returns once every rank has joined, or fails
        except (sh.SspError, TimeoutError) as e:
            err = e
        # Every rank agrees on the outcome through the launcher's file rendezvous (no collective of the
        # transport that may have failed).  If any rank's RCCL join failed, every rank attaches the host
        # hub in this same process (no re-exec, no restart): the run still yields a measured number, and
        # the JSON line names the transport that produced it.
        failed = agree_failures(rank, world, err)
        if uid_path:  # rank 0, once every rank has reported (so has read the id, or given up on it)
            os.remove(uid_path)
        if failed:
            log(f"rank {rank}: RCCL join failed on rank(s) {failed} ({err if err else 'this rank joined'}); "
                "every rank falls back to the host hub")
            port = int(os.environ.get("MASTER_PORT", "29500")) + 1
            ctx.attach_host_comm(sh.HubComm(rank, world, os.environ.get("MASTER_ADDR", "127.0.0.1"), port))
            transport = "host"
            args.comm_fallback = {"from": "rccl", "failed_ranks": failed,
                                  "reason": str(err) if err else f"RCCL join failed on rank(s) {failed}"}
    args.comm_used = transport
    return ctx


def agree_failures(rank, world, err, timeout=None):
    """The ranks whose attach failed, agreed by every rank: each writes its outcome to a file keyed by
    the launcher (as rendezvous_uid) and reads every rank's.  Bounded by SSP_COMM_TIMEOUT_S; a rank
    that never reports counts as failed."""
    timeout = float(os.environ.get("SSP_COMM_TIMEOUT_S", "120")) if timeout is None else timeout
    tag = "{}_{}_{}".format(os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                            os.getppid())
    base = os.path.join(tempfile.gettempdir(), f"ssp_bench_attach_{tag}")
    with open(f"{base}.{rank}.tmp", "w") as f:
        f.write("fail" if err else "ok")
    os.replace(f"{base}.{rank}.tmp", f"{base}.{rank}")
    t0, failed = time.time(), []
    for r in range(world):
        path = f"{base}.{r}"
        while not os.path.exists(path) and time.time() - t0 < timeout:
            time.sleep(0.05)
        try:
            with open(path) as f:
                ok = f.read() == "ok"
        except OSError:
            ok = False
        if not ok:
            failed.append(r)
    return failed


def remove_attach_files(world):
    """Rank 0, after the last barrier (every rank has read them): agree_failures' files."""
    tag = "{}_{}_{}".format(os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                            os.getppid())
    for r in range(world):
        try:
            os.remove(os.path.join(tempfile.gettempdir(), f"ssp_bench_attach_{tag}.{r}"))
        except OSError:
            pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    # not "--n": torch.distributed.run would take it as an abbreviation of its own --nnodes/--nproc-per-node
    ap.add_argument("--n-global", type=float, default=1e8, help="global vector length")
    ap.add_argument("--roots", type=int, default=8)
    ap.add_argument("--qsize", type=int, default=48)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-n", type=float, default=CPU_N, help="vector length of the 1-core CPU baseline step")
    ap.add_argument("--cpu-solve-n", type=float, default=C2_SOLVE["n"], help="length of the in-solver C2 solve")
    ap.add_argument("--ledger-steps", type=int, default=3,
                    help="with --no-timed-ledger: extra steps under the HIP-event ledger after the timed region")
    ap.add_argument("--no-timed-ledger", action="store_true",
                    help="time the K steps without HIP events (the roofline ledger then runs on --ledger-steps "
                         "extra steps); for measuring the events' cost")
    ap.add_argument("--no-in-solver", action="store_true", help="skip the whole-solve block")
    ap.add_argument("--no-small", action="store_true", help="skip the headline step at N / 10")
    ap.add_argument("--comm", choices=("rccl", "p2p", "auto", "host"), default="rccl",
                    help="rank transport at N > 1: RCCL; the peer-memory communicator (p2p: IPC-shared device "
                         "inboxes, rank-order sums); auto = p2p when its attach self-test passes on every rank, "
                         "else RCCL; or the host socket hub (tests: several ranks on ONE device)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r6", "pmc_traffic_n1e8_r6.json"),
                    help="rocprofv3 --pmc summary of this workload (roofline.traffic)")
    ap.add_argument("--mfma-json", default=os.path.join(ROOT, "profiles", "r3", "mfma_util_n1e8.json"),
                    help="rocprofv3 --pmc MfmaUtil summary of this workload (mfma.mfma_util_pct)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    t_ctx = time.perf_counter()
    try:
        ctx = setup_context(args, world, rank, local_rank)
    except Exception as e:  # noqa: BLE001 - a communicator that does not form ends the run with a record
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "higher_is_better": True, "rank": rank,
                          "error": f"communicator setup failed on rank {rank}: {e}"}), flush=True)
        sys.exit(3)

    ctx.synchronize()
    ctx_create_s = time.perf_counter() - t_ctx
    n_global = int(args.n_global)
    m, k = args.roots, args.qsize
    borders = distribution(n_global, world)
    n_local, offset = borders[rank + 1] - borders[rank], borders[rank]
    log(f"rank {rank}/{world}: n_local={n_local} vectors={2 * (m + k)} HBM={2 * (m + k) * n_local * 8 / 1e9:.1f} GB")
    wl = Workload(ctx, n_local, offset, m, k)

    def barrier():
        if world > 1:
            ctx.barrier()

    for _ in range(args.warmup):
        wl.step()
    ctx.synchronize()
    # The roofline ledger is the timed region itself: a HIP event pair on the context stream around
    # every op of the K steps (the kernels' own stream; resolved after the region).
    timed_ledger = not args.no_timed_ledger
    if timed_ledger:  # one counted step sizes the event pool: no event is created inside the region
        ctx.ledger_reset()
        ctx.ledger_enable(True)
        wl.step()
        ctx.ledger_enable(False)
        ctx.ledger_reserve(2 * sum(v["calls"] for v in ctx.ledger().values()) * args.steps)
        ctx.synchronize()
    ctx.ledger_reset()
    ctx.ledger_enable(timed_ledger)
    barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        wl.step()
    ctx.synchronize()
    t1 = time.perf_counter()
    ctx.ledger_enable(False)
    barrier()
    elapsed = t1 - t0
    if world > 1:  # max over ranks
        elapsed = max(struct.unpack("<d", b)[0] for b in ctx.allgather_bytes(struct.pack("<d", elapsed)))
    ledger_steps = args.steps
    if not timed_ledger:
        # Per-kernel HIP-event ledger over a few extra steps (not part of the timed region).
        ctx.ledger_reset()
        ctx.ledger_enable(True)
        for _ in range(args.ledger_steps):
            wl.step()
        ctx.ledger_enable(False)
        ledger_steps = args.ledger_steps
    led = ctx.ledger()

    # The product's own form of the same update (not the headline; see the module docstring).
    for _ in range(2):
        wl.product_step()
    ctx.synchronize()
    barrier()
    tp = time.perf_counter()
    p_steps = max(5, args.steps // 4)
    for _ in range(p_steps):
        wl.product_step()
    ctx.synchronize()
    tp = time.perf_counter() - tp
    if world > 1:
        tp = max(struct.unpack("<d", b)[0] for b in ctx.allgather_bytes(struct.pack("<d", tp)))
    ctx.ledger_reset()
    ctx.ledger_enable(True)
    wl.product_step()
    ctx.ledger_enable(False)
    pled = ctx.ledger()
    product = {
        "ms_per_step": round(1e3 * tp / p_steps, 4),
        "bytes_per_step": product_step_bytes(n_global, m, k),
        "GBs": round(product_step_bytes(n_global, m, k) * p_steps / tp / 1e9, 2),
        "vs_headline_step_time": None,
        "ops": {op: {"calls_per_step": v["calls"], "avg_us": round(1e3 * v["ms"] / v["calls"], 2),
                     "GBs": round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1)} for op, v in pled.items()},
    }
    # CPU baselines (rank 0 of a 1-GPU run) on ONE pinned host core, in a thread beside the GPU work
    # that follows (the reference loops release the GIL inside their C calls): the headline step's op
    # sequence at N = 1e7, DRAM-resident, then the C2 Davidson solve (BASELINE.md §3's "In-solver"
    # row).  Meanwhile the sustained phase repeats the headline step on the GPU for ~cpu_seconds -- its
    # long-run rate beside the timed region -- and the GPU solves run; host-parallel (all host threads)
    # and the DRAM-resident single calls come last, GPU idle.
    sustained, cb, th, box = None, None, None, {}
    run_cpu = world == 1 and not args.no_cpu_baseline
    if run_cpu:
        log("CPU baselines (oracle, 1 pinned core) in a thread beside the GPU work...")

        def cpu_leg():
            try:
                box["cb"] = cpu_baseline_core(m, k, args.cpu_seconds, int(args.cpu_n))
                box["solve"] = cpu_solve_core(args.cpu_solve_n)
            except Exception as e:  # noqa: BLE001 - reported in the JSON line, never fatal to the bench
                box["error"] = repr(e)

        th = threading.Thread(target=cpu_leg, daemon=True)
        ctx.synchronize()
        ts = time.perf_counter()
        th.start()
        n_sus = 0
        while n_sus < 5 or time.perf_counter() - ts < args.cpu_seconds:
            wl.step()
            n_sus += 1
        ctx.synchronize()
        ts = time.perf_counter() - ts
        sustained = {"steps": n_sus, "seconds": round(ts, 2), "ms_per_step": round(1e3 * ts / n_sus, 4),
                     "GBs": round(step_bytes(n_global, m, k) * n_sus / ts / 1e9, 2),
                     "note": "headline step repeated while the 1-core CPU baseline runs on another core"}
    wl.free()  # back to the arena before the whole solves
    # The same headline step at a tenth of the length (BASELINE config C2's N = 1e7 sharded alike):
    # the rate where launch and reduction latencies weigh ten times more.
    small = None
    if not args.no_small and n_global >= 10:
        ns_global = n_global // 10
        sb = distribution(ns_global, world)
        wls = Workload(ctx, sb[rank + 1] - sb[rank], sb[rank], m, k)
        for _ in range(3):
            wls.step()
        ctx.synchronize()
        barrier()
        t_s = time.perf_counter()
        s_steps = max(10, args.steps)
        for _ in range(s_steps):
            wls.step()
        ctx.synchronize()
        t_s = time.perf_counter() - t_s
        if world > 1:
            t_s = max(struct.unpack("<d", b)[0] for b in ctx.allgather_bytes(struct.pack("<d", t_s)))
        # its roofline as the headline's: the dominant op's average launch over a few ledgered steps
        # (HIP events on the context stream, after the timed region)
        ctx.ledger_reset()
        ctx.ledger_enable(True)
        for _ in range(5):
            wls.step()
        ctx.synchronize()
        ctx.ledger_enable(False)
        led_s = ctx.ledger()
        wls.free()
        dom_s = max(led_s, key=lambda op: led_s[op]["ms"])
        es = led_s[dom_s]
        ach_s = (es["bytes"] / es["calls"]) / (es["ms"] / es["calls"] / 1e3) / 1e9
        small = {"n_global": ns_global, "steps": s_steps, "ms_per_step": round(1e3 * t_s / s_steps, 4),
                 "GBs": round(step_bytes(ns_global, m, k) * s_steps / t_s / 1e9, 2),
                 "frac_of_hbm_peak": round(step_bytes(ns_global, m, k) * s_steps / t_s / 1e9 / HBM_PEAK_GBS, 4),
                 "roofline": {"bound": "hbm", "kernel": dom_s, "achieved": round(ach_s, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": float(f"{ach_s / HBM_PEAK_GBS:.4g}"),
                              "avg_launch_us": round(1e3 * es["ms"] / es["calls"], 2),
                              "bytes_per_launch": es["bytes"] / es["calls"],
                              "ledger": "HIP events over 5 steps after the timed region"}}
    solve = solve_diis = gpu_c2 = shard = None
    if not args.no_in_solver:
        solve = in_solver(ctx, n_global, world, barrier)
        solve_diis = in_solver(ctx, n_global, world, barrier, kind="diis")
        if world == 1 and n_global >= 8:
            # one rank's share of C4 (N / 8 elements, the same subspace work): the solve whose wall
            # against its kernel time bounds the 8-GPU C4 solve
            shard = in_solver(ctx, n_global // 8, world, barrier)
            shard["config"] = "C4, one rank's share on one GPU: " + shard["config"].split(": ", 1)[1]
        if run_cpu:
            gpu_c2 = gpu_c2_solve(ctx, world, args.cpu_solve_n)
    if th is not None:
        log("waiting for the CPU baselines...")
        th.join()
        cb = box.get("cb")

    total_bytes = step_bytes(n_global, m, k) * args.steps
    value = total_bytes / elapsed / 1e9
    result = None
    if rank == 0:
        dom = max(led, key=lambda op: led[op]["ms"])
        e = led[dom]
        achieved = (e["bytes"] / e["calls"]) / (e["ms"] / e["calls"] / 1e3) / 1e9
        traffic, traffic_src = pmc_traffic(args.pmc_json, dom, n_global, m, k, world)
        ops = {op: {"calls_per_step": v["calls"] / ledger_steps,
                    "avg_us": 1e3 * v["ms"] / v["calls"],
                    "GBs": v["bytes"] / (v["ms"] / 1e3) / 1e9} for op, v in led.items()}
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 uniform [-1,1), global-index seeded; HBM-resident)",
            "config": {
                "workload": "Davidson subspace update per step: 2x gemm_inner(8x48) + 2x construct_solution "
                            "(fill x8 + gemm_outer 48->8) + 8x residual axpy + 8x norm dot",
                "n_global": n_global,
                "n_local_rank0": n_local,
                "roots": m,
                "qspace": k,
                "parallelism": f"index-range shards x{world} ("
                               + {"rccl": "RCCL", "p2p": "peer-memory", "host": "host-hub"}[getattr(args, "comm_used", args.comm)]
                               + " allreduce for reductions)",

                "bytes_per_step": step_bytes(n_global, m, k),
            },
            "comm": getattr(args, "comm_used", args.comm) if world > 1 else None,
            "comm_fallback": getattr(args, "comm_fallback", None),
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": float(f"{achieved / HBM_PEAK_GBS:.4g}"),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_launch_us": round(1e3 * e["ms"] / e["calls"], 2),
                "bytes_per_launch": e["bytes"] / e["calls"],
            },
            "ops": ops,
            "ledger": "HIP events around every op of the timed steps" if timed_ledger
                      else f"HIP events over {ledger_steps} extra steps after the timed region",
            "product_step": product,
            "headline_step_at_n_div_10": small,
            "in_solver": solve,
            "in_solver_diis": solve_diis,
            "in_solver_c4_shard": shard,
            "startup": {"ctx_create_s": round(ctx_create_s, 3),
                        "first_solve_wall_s": solve["wall_s_cold"] if solve else None,
                        "warm_solve_wall_s": solve["wall_s"] if solve else None},
        }
        product["vs_headline_step_time"] = round(product["ms_per_step"] / (1e3 * elapsed / args.steps), 4)
        if "gemm_inner" in led and world == 1:
            # gemm_inner runs on the f64 matrix cores: live MFMA rate from the ledger (2 m k N flops
            # per call) against the dense f64 MFMA peak, and the PMC-measured MfmaUtil beside it.
            gi = led["gemm_inner"]
            tflops = 2.0 * m * k * n_local * gi["calls"] / (gi["ms"] / 1e3) / 1e12
            util, util_src = mfma_util(args.mfma_json)
            result["mfma"] = {"kernel": "gemm_inner", "achieved_tflops": round(tflops, 2),
                              "peak_tflops": MFMA_F64_PEAK_TFLOPS, "frac": round(tflops / MFMA_F64_PEAK_TFLOPS, 4),
                              "mfma_util_pct": util, "util_source": util_src}
        if cb is not None:
            cpu_baseline_extras(cb, m, k, args.cpu_seconds)
        result["cpu_baseline"] = cb
        if run_cpu:
            cs = box.get("solve")
            result["in_solver_cpu"] = {
                "config": f"LinearEigensystemDavidson C2 (BASELINE.md §3 In-solver): 4 roots, N={args.cpu_solve_n:.0e}, rank-one "
                          "H = diag(1+i) + 0.1 1 1^T, max_size_qspace 24, reset_D 8, threshold 1e-8",
                "cpu": cs, "gpu": gpu_c2, "cpu_path_trace": "tests/golden/traces.json:C2_rank1",
                "speedup": round(cs["wall_s"] / gpu_c2["wall_s"], 1) if cs and gpu_c2 else None,
                "same_iterations": bool(cs and gpu_c2 and cs["iterations"] == gpu_c2["iterations"]),
                "error": box.get("error")}
        result["sustained"] = sustained
        print(json.dumps(result), flush=True)
    barrier()
    if rank == 0 and world > 1:
        remove_attach_files(world)
    ctx.close()
    if getattr(args, "comm_fallback", None):
        # an abandoned RCCL join leaves its helper thread inside RCCL's bootstrap: end the process
        # without the interpreter's teardown (the JSON line is out)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
