#!/bin/bash
# Round-4 GPU session T (final tree): the whole GPU suite (verbose, slowest tests listed), smoke, the
# bench and its rocprofv3 kernel statistics.  A heartbeat line per minute under gpurun_out/ marks
# the long multi-process tests as alive; each test still has its own 600 s limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R4T_OUT:-r4t}
mkdir -p "$OUT"
export TMPDIR=/tmp
(while sleep 60; do date +%T >> "$OUT/heartbeat"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step gpu_suite 1500 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread -rf --durations=12 || exit $?
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
step bench 900 python -u bench.py || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
rm -rf "$OUT/prof"
step bench_rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 || exit $?
grep '^{' "$OUT/bench_rocprof.log" > "$OUT/bench_under_rocprof.json" || true
echo "session done"
