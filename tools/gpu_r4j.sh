#!/bin/bash
# Round-4 GPU session J: batched sparse axpy test, C4-shard ledger and kernel trace (synthetic action
# kernels with compile-time vector groups).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4j
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step tests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_solver_gpu.py tests/test_traces_gpu.py -q -x --timeout 200 --timeout-method thread -rf -k "sparse or synthetic or davidson or trace" || exit $?
step exact_cost 300 python -u tools/exact_cost.py --out "$OUT/exact_cost.json" || exit $?
step transport_ab 600 python -u tools/transport_ab.py --config C4-shard --reps 5 --out "$OUT/transport_ab_c4shard.json" || exit $?
step ledger 600 python -u tools/solver_ledger.py --configs C3,C4-shard --out "$OUT/solver_ledger.json" || exit $?
rm -rf "$OUT/trace"
step trace 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
  python3 tools/solver_ledger.py --configs C4-shard --out "$OUT/ledger_traced.json" || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$OUT/pmc_$c"
  step "pmc_$c" 300 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- \
    python3 tools/solver_ledger.py --configs C4-shard --out "$OUT/ledger_pmc_$c.json" || exit $?
done
python3 tools/pmc_solve_summary.py "$(dirname "$(find "$OUT/pmc_FETCH_SIZE" -name '*counter_collection.csv' | head -1)")" \
  "$(dirname "$(find "$OUT/pmc_WRITE_SIZE" -name '*counter_collection.csv' | head -1)")" "$OUT/ledger_pmc_FETCH_SIZE.json" \
  "$OUT/pmc_c4shard.json" > /dev/null || true
echo "session done"
