"""Writes tests/golden/mpich_traces.json: the short synthetic solves of make_traces.py MPI_CASES run by
the CPU path -- the product's host code over the host-memory emulation (oracle/ssp_emul.cpp), each
rank's dots the reference's sequential loop -- sharded over P = 2, 3, 4, 8 MPI ranks under this
container's MPICH (`mpiexec -n P`, /opt/conda MPICH 3.3.2), the ranks' partials summed by MPICH's own
MPI_Allreduce (the "mpi" transport of iterative-solver_amd/host/mpi_bridge.h): the reference's
distributed build's reduction (DistrArray.cpp:133-135, util/gemm.h:179-182) with a real MPI library's
association, not a modelled one.

Then checks, in this process, that the restated CPU path with its dots summed by the association
model oracle_ops.c sum order 200 + P reproduces every record bit for bit (and reports where the
rank-order sums of mpi_traces.json differ).

    python tests/golden/make_mpi_traces.py       (after `make -C oracle`)
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "mpich_traces.json")
MPIEXEC = os.environ.get("MPIEXEC", "/opt/conda/bin/mpiexec")
WORLDS = (2, 3, 4, 8)


def main():
    if os.path.exists(OUT):
        os.remove(OUT)
    for p in WORLDS:
        r = subprocess.run([MPIEXEC, "-n", str(p), sys.executable, os.path.join(ROOT, "tests", "mpi_worker.py"), "synth",
                            "emul", "mpi", "record", OUT], capture_output=True, text=True, timeout=1200,
                           env=dict(os.environ, OMP_NUM_THREADS="1"))
        print(r.stdout.strip(), flush=True)
        if r.returncode != 0:
            raise SystemExit(r.stdout[-3000:] + r.stderr[-3000:])
    rec = json.load(open(OUT))
    sys.path.insert(0, HERE)
    from make_traces import ORACLE_REVISION

    rec["_parity"] = "bit_exact"
    rec["_oracle_revision"] = ORACLE_REVISION
    rec["_generator"] = ("tests/golden/make_mpi_traces.py: CPU path (product host code over oracle/ssp_emul.cpp, "
                         "sequential rank-local dots) under mpiexec -n P of /opt/conda MPICH 3.3.2, rank partials "
                         "summed by MPI_Allreduce(MPI_SUM)")
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), HERE]
    import numpy as np

    import oracle
    from make_traces import MPI_CASES, mpi_options

    ranko = json.load(open(os.path.join(HERE, "mpi_traces.json")))
    for name, c in MPI_CASES.items():
        fn = oracle.davidson_synthetic if c["kind"] == "davidson" else oracle.diis_synthetic
        for p in WORLDS:
            oracle.set_sum_order(200 + p)
            r = fn(c["n"], c["rho"], c["rank"], c["seed"], solutions=False, **mpi_options(c))
            got = rec[name][f"mpich{p}"]
            for f in ("iterations", "r_creations", "q_creations"):
                assert r[f] == got[f], (name, p, f, r[f], got[f])
            for f in ("eigenvalues", "errors"):
                assert [float(x) for x in r[f]] == got[f], (name, p, f)
            for f in ("eigenvalues", "errors", "nq", "nwork", "screened"):
                assert np.asarray(r["trace"][f]).tolist() == got["trace"][f], (name, p, "trace", f)
            same = ranko[name].get(f"mpi{p}", {}).get("trace") == got["trace"]
            print(f"{name} P={p}: {got['iterations']} iterations; model 200+{p} bit-identical; rank-order sums "
                  f"{'identical' if same else 'differ'}", flush=True)
        oracle.set_sum_order(0)
    json.dump(rec, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
