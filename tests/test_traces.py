"""The committed per-iteration traces of the reference CPU path (tests/golden/traces.json,
tests/golden/make_traces.py): C1 (N = 1e4, 1 root -- BASELINE config 1, the CPU
ArrayHandlerIterable plumbing case) is re-run here and must reproduce its trace bit for bit (the CPU
path is deterministic), and every rank-1 trace must end on the exact eigenvalues of
diag(1 + i) + rho 11^T (secular equation), which pins the fixtures independently of the oracle."""
import json
import os

import numpy as np
import pytest

import oracle

T = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "traces.json")))


@pytest.mark.parametrize("name", ["C1_rank1", "C1_rank8"])
def test_c1_cpu_path_reproduces_trace(name):
    ref = T[name]
    c = ref["case"]
    r = oracle.davidson_synthetic(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **ref["options"])
    assert r["converged"] and r["iterations"] == ref["iterations"] and r["r_creations"] == ref["r_creations"]
    assert r["trace"]["eigenvalues"].tolist() == ref["trace"]["eigenvalues"]
    assert r["trace"]["errors"].tolist() == ref["trace"]["errors"]
    assert r["trace"]["nq"].tolist() == ref["trace"]["nq"]


@pytest.mark.parametrize("name", sorted(k for k, v in T.items() if not k.startswith("_")
                                        and v["case"]["kind"] == "davidson" and v["case"]["rank"] == 1))
def test_rank_one_traces_end_on_exact_eigenvalues(name):
    ref = T[name]
    c = ref["case"]
    assert ref["converged"]
    exact = oracle.rank_one_eigenvalues(c["n"], c["rho"], c["nroots"])
    np.testing.assert_allclose(ref["eigenvalues"], exact, rtol=1e-10, atol=0)
    assert max(ref["errors"]) <= 1e-8


def test_traces_cover_the_baseline_configs():
    # C1, C2, C3 (shape at 1e7 and the real size at 1e8), C5 (the well-posed instance at 1e7 and 1e8;
    # the round-1 chaotic instance C5x as its 12-iteration descent + converged run)
    for k in ("C1_rank1", "C2_rank1", "C2_rank8", "C3_n1e7_rank8", "C3_n1e8_rank1", "C3_n1e8_rank8", "C5_n1e7",
              "C5_n1e8", "C5x_n1e7_traj12", "C5x_n1e7"):
        assert k in T
    # the bench's own solve at full size (bench.py in_solver, C4's problem): the full trace bar applies
    # (the CPU path takes the same steps under both reordered sums)
    c3 = T["C3_n1e8_rank8"]
    assert c3["case"]["n"] == 100_000_000 and c3["case"]["rank"] == 8 and c3["options"]["max_p"] == 16
    assert c3["options"]["max_size_qspace"] == 48 and c3["converged"]
    assert c3["reordered"]["same_steps"] and c3["reordered_blocked"]["same_steps"]
    assert T["C3_n1e8_rank1"]["case"]["n"] == 100_000_000 and T["C3_n1e8_rank1"]["options"]["max_p"] == 16
    assert T["C2_rank8"]["options"]["nroots"] == 4 and T["C2_rank8"]["case"]["n"] == 10_000_000


@pytest.mark.parametrize("name", ["C5_n1e7", "C5_n1e8"])
def test_c5_traces_are_well_posed(name):
    # C5's parity observables are not decided by rounding: the CPU path takes the same steps when only
    # its summation order changes (make_traces.py "reordered" and "reordered_blocked"), it converges,
    # every error it
    # decides on lies at least 20 % away from the threshold (no knife edge), while the rounding floor
    # eps |r_0| sits four orders below it.
    ref = T[name]
    assert ref["converged"]
    for v in ("reordered", "reordered_blocked"):
        assert ref[v]["same_steps"] and ref[v]["converged"], v
    assert ref["iterations"] >= 8 and ref["r_creations"] == ref["iterations"] + 1
    e = np.array(ref["trace"]["errors"])[:, 0]
    thr = ref["options"]["convergence_threshold"]
    assert np.all(np.abs(e / thr - 1.0) > 0.2)
    assert 2.2e-16 * e[0] < 1e-3 * thr
    assert e[-1] < thr and np.all(e[:-1] > thr)


_OMP_CASE = r"""
import json, sys
sys.path[:0] = sys.argv[1:3]
import oracle
out = {}
for order in (0, 2):
    oracle.set_sum_order(order)
    r = oracle.davidson_synthetic(300_000, 0.1, 8, 1, solutions=False, nroots=4, max_p=4, convergence_threshold=1e-8,
                                  max_size_qspace=24, reset_D=8)
    out[order] = [r["iterations"], r["r_creations"], r["trace"]["eigenvalues"].tolist(), r["trace"]["errors"].tolist(),
                  r["trace"]["nq"].tolist()]
print(json.dumps(out))
"""


def test_openmp_oracle_is_bit_identical_to_the_sequential_cpu_path():
    # make_traces.py --omp (the C3_n1e8_rank8 trace, ~100 GB) runs the CPU path with its independent
    # elements on several threads (oracle/build/liboracle_itsolv_omp.so): every number must equal the
    # sequential build's, in the reference order and in the blocked reordering
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    paths = [os.path.join(root, "iterative-solver_amd"), os.path.join(root, "oracle")]
    if not os.path.exists(os.path.join(root, "oracle", "build", "liboracle_itsolv_omp.so")):
        subprocess.run(["make", "-C", os.path.join(root, "oracle")], check=True, capture_output=True)
    runs = []
    for omp in ("0", "1"):
        env = dict(os.environ, ORACLE_OMP=omp, OMP_NUM_THREADS="4")
        r = subprocess.run([sys.executable, "-c", _OMP_CASE, *paths], env=env, capture_output=True, text=True,
                           timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        runs.append(r.stdout)
    assert runs[0] == runs[1]


def test_fixture_parity_classes_and_revisions():
    # Every committed trace says what it pins and which oracle revision wrote it (make_traces.py
    # BIT_EXACT / ORACLE_REVISION): the bit-exact fixtures (C1, and every record of mpi_traces.json and
    # mpich_traces.json) carry the current revision of the shared host algebra; the tolerance traces
    # (N >= 2^21) may carry an older one, which their bar absorbs.
    import sys

    golden = os.path.join(os.path.dirname(__file__), "golden")
    sys.path.insert(0, golden)
    from make_traces import BIT_EXACT, ORACLE_REVISION

    for name, rec in T.items():
        if name.startswith("_"):
            continue
        assert rec["parity"] == ("bit_exact" if name in BIT_EXACT else "tolerance"), name
        assert rec["oracle_revision"].split(":")[0] in ("r5",), name
        if rec["parity"] == "bit_exact":
            assert rec["oracle_revision"] == ORACLE_REVISION, name
        else:
            assert rec["case"]["n"] >= 1 << 21, name
    for f in ("mpi_traces.json", "mpich_traces.json"):
        d = json.load(open(os.path.join(golden, f)))
        assert d["_parity"] == "bit_exact" and d["_oracle_revision"] == ORACLE_REVISION, f
