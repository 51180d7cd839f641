#!/bin/bash
# Round-4 GPU session L: SURVEY.md §8d per-shape microbenchmark at N = 1e8 and 1e7 (median of 10
# repetitions).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4l
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step shapes_1e8 600 python -u tools/shapes_bench.py --n 1e8 --reps 10 --out "$OUT/shapes_n1e8.json" || exit $?
step shapes_1e7 300 python -u tools/shapes_bench.py --n 1e7 --reps 10 --out "$OUT/shapes_n1e7.json" || exit $?
echo "session done"
