#!/bin/bash
# Round-4 GPU session O: the size-selected synthetic apply shape -- tests, C3 / C4-shard ledgers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4o
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-220; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step tests 900 python -u -m pytest tests/test_ops_gpu.py tests/test_traces_gpu.py tests/test_exact_gpu.py tests/test_solver_gpu.py tests/test_scaled_gpu.py -q -x --timeout 200 --timeout-method thread -rf || exit $?
step dist 900 python -u -m pytest tests/test_distributed_gpu.py -q -x --timeout 600 --timeout-method thread -rf -k "traces or mpi_build or solver" || exit $?
step ledger_1 300 python -u tools/solver_ledger.py --configs C3,C4-shard,C5 --out "$OUT/ledger_1.json" || exit $?
step ledger_2 300 python -u tools/solver_ledger.py --configs C3,C4-shard,C5 --out "$OUT/ledger_2.json" || exit $?
echo "session done"
