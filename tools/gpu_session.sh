#!/bin/bash
# One GPU-box session: any of the GPU tests, smoke, bench, kernel-trace profile, PMC passes, ledgers.
#
#   tools/gpu_session.sh STEPS [args...]      STEPS: comma-separated, run in order, e.g. tests,smoke,bench
#     tests   [pytest args]   python -m pytest tests -m gpu -v (every test named as it starts and ends)
#     smoke                    __graft_entry__.smoke()
#     bench   [bench args]     python bench.py
#     prof    [bench args]     rocprofv3 --kernel-trace --stats of a short bench run
#     pmc     [bench args]     HBM traffic counters (FETCH_SIZE, WRITE_SIZE), one --pmc pass each
#     mfma    [bench args]     matrix-core counters of the bench step and of the per-shape bench
#     ledger                   tools/shapes_bench.py and tools/solver_ledger.py
#   Outputs: gpurun_out/${SESSION:-session}/<step>.log (+ bench.json, prof/, pmc_*/).
#
# Every step streams its output to stdout (tee) as well as to its log, and a heartbeat line goes to
# stdout every 50 s: the pool takes a command that is silent on stdout / stderr / gpurun_out for 180 s
# as hung and kills it, and a single long test (the 8-process full-size solves) prints nothing while it
# runs.  Each step has its own time limit; a fault, abort or timeout ends the session (no retries).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${SESSION:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
steps=${1:-tests,smoke,bench,prof}
shift || true

(while sleep 50; do echo "[heartbeat $(date +%T)]"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT

step() {  # step <name> <seconds> <cmd...>: the command's status; output to stdout and $OUT/<name>.log
  local name=$1 t=$2
  shift 2
  echo "== $name (limit ${t}s): $*"
  timeout -k 10 "$t" "$@" 2>&1 | tee "$OUT/$name.log"
  local rc=$?
  echo "== $name rc=$rc"
  return $rc
}

for s in ${steps//,/ }; do
  case $s in
    tests)
      step pytest_gpu 2400 python -u -m pytest tests -m gpu -v -x -rf --durations=15 --timeout 600 \
        --timeout-method thread "$@" || exit $?
      ;;
    smoke)
      step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
      ;;
    bench)
      step bench 900 python -u bench.py "$@" || exit $?
      grep '^{' "$OUT/bench.log" >"$OUT/bench.json" || true
      ;;
    prof)
      rm -rf "$OUT/prof"
      step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" || exit $?
      # the bench line of the profiled process itself: its ledger and the kernel statistics come
      # from the same allocation
      grep '^{' "$OUT/rocprof.log" >"$OUT/bench_rocprof.json" || true
      ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf "$OUT/pmc_$c"
        step "pmc_$c" 600 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- \
          python3 bench.py --steps 2 --warmup 1 --ledger-steps 1 --no-cpu-baseline --no-in-solver --no-small \
          "$@" || exit $?
      done
      ;;
    mfma)
      rm -rf "$OUT/pmc_mfma" "$OUT/pmc_mfma_shapes"
      step pmc_mfma 600 rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 --kernel-trace \
        -d "$OUT/pmc_mfma" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --ledger-steps 1 \
        --no-cpu-baseline --no-in-solver --no-small "$@" || exit $?
      step pmc_mfma_shapes 600 rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 --kernel-trace \
        -d "$OUT/pmc_mfma_shapes" -o run --output-format csv -- python3 tools/shapes_bench.py --reps 1 \
        --out "$OUT/shapes_pmc.json" || exit $?
      ;;
    ledger)
      step shapes 600 python -u tools/shapes_bench.py --out "$OUT/shapes.json" || exit $?
      step solver_ledger 900 python -u tools/solver_ledger.py --out "$OUT/solver_ledger.json" || exit $?
      ;;
    *)
      echo "unknown step $s"
      exit 2
      ;;
  esac
done
echo "session done"
