#!/bin/bash
# Round-4 GPU session A: new comm tests (deadline, one-rank p2p, multi-rank p2p, lost rank), the
# near-dependent RS traces, and the reduction-latency / C4-shard ledgers on RCCL vs p2p.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4a
mkdir -p "$OUT"
export TMPDIR=/tmp
# a step's status: 0 ok, 1 test failures (go on), anything else (timeout, abort, fault) ends the session
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step p2p_dist 900 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 300 --timeout-method thread -k "p2p or lost_rank" || exit $?
step lat_rccl 300 python -u tools/latency_probe.py --rccl --out "$OUT/latency_rccl.json" || exit $?
step lat_p2p 300 python -u tools/latency_probe.py --p2p --out "$OUT/latency_p2p.json" || exit $?
step lat_fused 300 python -u tools/latency_probe.py --out "$OUT/latency_fused.json" || exit $?
step ledger_rccl 300 python -u tools/solver_ledger.py --configs C4-shard --rccl --out "$OUT/ledger_c4shard_rccl.json" || exit $?
step ledger_p2p 300 python -u tools/solver_ledger.py --configs C4-shard --p2p --out "$OUT/ledger_c4shard_p2p.json" || exit $?
step ledger_c3 300 python -u tools/solver_ledger.py --configs C3,C5 --out "$OUT/ledger_c3_c5.json" || exit $?
# kernel timelines of the C4-shard solve (idle gaps: tools/gap_analysis.py)
for t in rccl p2p; do
  rm -rf "$OUT/trace_$t"
  step "trace_$t" 300 rocprofv3 --kernel-trace -d "$OUT/trace_$t" -o run --output-format csv -- \
    python3 tools/solver_ledger.py --configs C4-shard --$t --out "$OUT/ledger_c4shard_${t}_traced.json" || exit $?
  python3 tools/gap_analysis.py "$(find "$OUT/trace_$t" -name '*kernel_trace.csv' | head -1)" --out "$OUT/gaps_c4shard_$t.json" > /dev/null
done
echo "session done"
