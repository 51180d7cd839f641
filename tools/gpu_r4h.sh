#!/bin/bash
# Round-4 GPU session H: exact-mode kernels pipelined / inline -- parity and cost.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4h
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step exact_tests 600 python -u -m pytest tests/test_exact_gpu.py tests/test_fortran.py tests/test_solver_gpu.py -q -x --timeout 120 --timeout-method thread -rf || exit $?
step exact_cost 300 python -u tools/exact_cost.py --out "$OUT/exact_cost.json" || exit $?
echo "session done"
