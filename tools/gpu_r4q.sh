#!/bin/bash
# Round-4 GPU session Q: the 8 x 48 overlap panel on different vector sets (role vs placement).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4q
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "gemm_inner 8x48\|gemm_inner 48x8" "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
for rep in 1 2; do
  for n in 1e7 1e8; do
    step "shapes_${n}_$rep" 600 python -u tools/shapes_bench.py --n $n --reps 10 --out "$OUT/shapes_${n}_$rep.json" || exit $?
  done
done
echo "session done"
