#!/bin/bash
# Round-4 GPU session D: the reference arithmetic on short vectors (kernels_exact.hip) -- bitwise
# parity tests, then the suites whose short-vector solves it changes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4d
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step exact_tests 300 python -u -m pytest tests/test_exact_gpu.py -q --timeout 120 --timeout-method thread -rf || exit $?
step solver_tests 900 python -u -m pytest tests/test_ops_gpu.py tests/test_scaled_gpu.py tests/test_solver_gpu.py tests/test_traces_gpu.py tests/test_fortran.py tests/test_python_api_gpu.py tests/test_reverse_comm.py -q --timeout 200 --timeout-method thread -rf || exit $?
echo "session done"
