#!/bin/bash
# Round-4 GPU session I: the 2048-element default -- exact parity suites and the sharded MPI-build runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4i
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step tests 900 python -u -m pytest tests/test_exact_gpu.py tests/test_fortran.py tests/test_ops_gpu.py tests/test_python_api_gpu.py tests/test_reverse_comm.py tests/test_solver_gpu.py -q -x --timeout 200 --timeout-method thread -rf || exit $?
step mpi 600 python -u -m pytest tests/test_distributed_gpu.py -k "mpi_build" -q -x --timeout 300 --timeout-method thread -rf || exit $?
echo "session done"
