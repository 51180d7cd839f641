#!/bin/bash
# Round-4 GPU session H: exact-mode kernels pipelined / inline, synthetic action kernels with
# compile-time vector groups -- parity, cost and the C3 / C4-shard ledgers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4h
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step tests 900 python -u -m pytest tests/test_exact_gpu.py tests/test_ops_gpu.py tests/test_scaled_gpu.py tests/test_fortran.py tests/test_solver_gpu.py tests/test_traces_gpu.py -q -x --timeout 200 --timeout-method thread -rf || exit $?
step exact_cost 300 python -u tools/exact_cost.py --out "$OUT/exact_cost.json" || exit $?
step ledger 600 python -u tools/solver_ledger.py --configs C3,C4-shard --out "$OUT/solver_ledger.json" || exit $?
echo "session done"
