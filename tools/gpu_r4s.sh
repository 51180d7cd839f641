#!/bin/bash
# Round-4 GPU session S: the inline sparse inner products publish from their last workgroup (and
# their ledger scope closes before the host wait) -- the suites through it, then the solve ledgers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4s
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"; return $rc; }
step tests 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu -k "not full_size" \
  tests/test_exact_gpu.py tests/test_fortran.py tests/test_reverse_comm.py tests/test_python_api_gpu.py \
  tests/test_ops_gpu.py tests/test_solver_gpu.py tests/test_distributed_gpu.py || exit $?
step ledger_1 300 python -u tools/solver_ledger.py --configs C3,C4-shard,C5 --out "$OUT/ledger_1.json" || exit $?
step ledger_2 300 python -u tools/solver_ledger.py --configs C3,C4-shard,C5 --out "$OUT/ledger_2.json" || exit $?
echo "session done"
