#!/bin/bash
# Round-4 GPU session N: synthetic apply kernel, window shape (default) vs the grid-strided pipelined
# form (SSP_SYNTH_SHAPE=stride): C3 / C4-shard ledgers, alternating; traces hold the results.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4n
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-220; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step tests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_traces_gpu.py tests/test_exact_gpu.py -q -x --timeout 200 --timeout-method thread -rf -k "synthetic or trace or davidson or diis or sparse" || exit $?
for rep in 1 2; do
  step "ledger_win_$rep" 300 python -u tools/solver_ledger.py --configs C3,C4-shard --out "$OUT/ledger_win_$rep.json" || exit $?
  SSP_SYNTH_SHAPE=stride step "ledger_stride_$rep" 300 python -u tools/solver_ledger.py --configs C3,C4-shard --out "$OUT/ledger_stride_$rep.json" || exit $?
done
echo "session done"
