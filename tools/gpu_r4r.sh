#!/bin/bash
# Round-4 GPU session R: the short-vector dot with the host publish fused into k_exact_inner --
# every bit-for-bit suite that runs through it, then the exact-path cost.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4r
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"; return $rc; }
step exact_tests 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu -k "not full_size" \
  tests/test_exact_gpu.py tests/test_fortran.py tests/test_reverse_comm.py tests/test_python_api_gpu.py \
  tests/test_ops_gpu.py tests/test_solver_gpu.py tests/test_distributed_gpu.py || exit $?
step exact_cost 300 python -u tools/exact_cost.py || exit $?
echo "session done"
