#!/bin/bash
# One GPU-box session: GPU tests, bench, kernel-trace profile.  Each GPU step has its own time limit;
# a fault / abort / timeout ends the session (no retries).  Outputs land in gpurun_out/.
# Usage: tools/gpu_session.sh [tests|bench|prof|pmc|mfma|ledger|all] [extra bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
what=${1:-all}
shift || true

step() {  # step <name> <seconds> <cmd...>; returns the command's status
  local name=$1 t=$2
  shift 2
  echo "== $name (limit ${t}s): $*"
  timeout -k 10 "$t" "$@" >"$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  return $rc
}

fatal() {  # statuses after which nothing else may use the GPU in this call
  case $1 in 0 | 1) return 1 ;; *) return 0 ;; esac
}

if [ "$what" = tests ] || [ "$what" = all ]; then
  step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread
  rc=$?
  if fatal $rc; then exit $rc; fi
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  step bench 900 python bench.py "$@"
  rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep '^{' "$OUT/bench.log" >"$OUT/bench.json" || true
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  rm -rf "$OUT/prof"
  step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-in-solver --no-small "$@"
  rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
  # The bench line of the profiled process itself: its HIP-event ledger and the kernel statistics
  # below come from the same allocation (placement moves gemm_outer by up to 8 % between processes).
  grep '^{' "$OUT/rocprof.log" >"$OUT/bench_rocprof.json" || true
fi
if [ "$what" = pmc ] || [ "$what" = all ]; then
  # HBM traffic counters, one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass);
  # kernel trace only, no runtime/API tracing alongside --pmc.
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf "$OUT/pmc_$c"
    step "pmc_$c" 600 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --ledger-steps 1 --no-cpu-baseline --no-in-solver --no-small "$@"
    rc=$?
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
fi
if [ "$what" = mfma ] || [ "$what" = all ]; then
  # Matrix-core activity (MfmaUtil, MfmaFlopsF64): the bench step, then the per-shape bench
  # (gemm_inner 16x64 is the densest panel), one --pmc pass each.
  rm -rf "$OUT/pmc_mfma" "$OUT/pmc_mfma_shapes"
  step pmc_mfma 600 rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 --kernel-trace -d "$OUT/pmc_mfma" \
    -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --ledger-steps 1 --no-cpu-baseline --no-in-solver --no-small "$@"
  rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
  step pmc_mfma_shapes 600 rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 --kernel-trace \
    -d "$OUT/pmc_mfma_shapes" -o run --output-format csv -- python3 tools/shapes_bench.py --reps 1 \
    --out "$OUT/shapes_pmc.json"
  rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "$what" = ledger ] || [ "$what" = all ]; then
  step shapes 600 python tools/shapes_bench.py --out "$OUT/shapes.json"
  rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
  step solver_ledger 900 python tools/solver_ledger.py --out "$OUT/solver_ledger.json"
  rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
echo "session done"
