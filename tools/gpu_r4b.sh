#!/bin/bash
# Round-4 GPU session B: sharded traces (host and peer-memory transports, RS cases included), the RS
# traces with both orthonormalisation forms, the lost-rank tests, the transport A/B, and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4b
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step pytest_gpu 1100 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread || exit $?
step lat_rccl 300 python -u tools/latency_probe.py --rccl --out "$OUT/latency_rccl.json" || exit $?
step lat_p2p 300 python -u tools/latency_probe.py --p2p --out "$OUT/latency_p2p.json" || exit $?
step transport_ab 600 python -u tools/transport_ab.py --config C4-shard --reps 5 --out "$OUT/transport_ab_c4shard.json" || exit $?
step bench 900 python -u bench.py || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
echo "session done"
