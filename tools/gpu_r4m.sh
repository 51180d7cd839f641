#!/bin/bash
# Round-4 GPU session M: gemm_inner workgroups per CU at N = 1e7 / 1.25e7 / 1e8 (SSP_INNER_PER_CU A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4m
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "gemm_inner 8x48\|gemm_inner 16x64\|gemm_inner 48x8" "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
for pc in 4 2 8 16 4; do
  for n in 1e7 1.25e7; do
    SSP_INNER_PER_CU=$pc step "inner_pc${pc}_n${n}" 300 python -u tools/shapes_bench.py --n $n --reps 10 --out "$OUT/shapes_pc${pc}_n${n}.json" || exit $?
  done
done
echo "session done"
