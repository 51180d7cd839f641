#!/bin/bash
# Round-4 GPU session C: C4-shard idle after the host-algebra and upload changes (transport A/B),
# solver ledgers, and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step ops_tests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_scaled_gpu.py tests/test_traces_gpu.py tests/test_rccl_gpu.py tests/test_solver_gpu.py -x -q --timeout 200 --timeout-method thread || exit $?
step dist_tests 600 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread -k "ops or distr or solver" || exit $?
step transport_ab 600 python -u tools/transport_ab.py --config C4-shard --reps 5 --out "$OUT/transport_ab_c4shard.json" || exit $?
step ledger 600 python -u tools/solver_ledger.py --configs C3,C5,C4-shard --out "$OUT/solver_ledger.json" || exit $?
rm -rf "$OUT/trace_p2p"
step trace_p2p 300 rocprofv3 --kernel-trace -d "$OUT/trace_p2p" -o run --output-format csv -- \
  python3 tools/solver_ledger.py --configs C4-shard --p2p --out "$OUT/ledger_c4shard_p2p_traced.json" || exit $?
python3 tools/gap_analysis.py "$(find "$OUT/trace_p2p" -name '*kernel_trace.csv' | head -1)" --span-ms 55 --out "$OUT/gaps_c4shard_p2p.json" > /dev/null
echo "session done"
