#!/bin/bash
# Round-6 GPU session steps: the default bench, the C4-shard solve ledger (per-instance rows and the
# host algebra clock), and a kernel trace of the C4-shard solve.
#   tools/gpu_r6.sh STEPS     STEPS: comma-separated of bench,benchprof,mergeab,synthtests,shapes,smoke,pmcbench,pmcc4,shapetab,selkern,c4ledger,c4pipe2,c4prof,c4trace,c4hiptrace,gapprobe,sizeprobe,seltests,selprobe,innertests,csab,outercu,outerab,selsizes,kernargab,kernargab2,fusedab,gputests
# Outputs under gpurun_out/${SESSION:-r6}/.  Each step has its own time limit; the first failure ends
# the session.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r6}
mkdir -p "$OUT"
export TMPDIR=/tmp
(while sleep 50; do echo "[heartbeat $(date +%T)]"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name (limit ${t}s): $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
for s in ${1//,/ }; do
  case $s in
    bench)
      step bench 600 python -u bench.py || exit $?
      grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
      ;;
    c4ledger)
      SSP_LEDGER_DETAIL=1 step c4ledger 300 python -u tools/solver_ledger.py --configs C4-shard,C3,C5 \
        --out "$OUT/c4_ledger.json" || exit $?
      ;;
    c4pipe2)
      SSP_INNER_PIPE=2 SSP_LEDGER_DETAIL=1 step c4pipe2 300 python -u tools/solver_ledger.py --configs C4-shard \
        --out "$OUT/c4_ledger_pipe2.json" || exit $?
      ;;
    seltests)
      step seltests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "select" \
        tests/test_ops_gpu.py tests/test_fullsize_gpu.py tests/test_distributed_gpu.py tests/test_rccl_gpu.py || exit $?
      ;;
    innertests)
      step innertests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "gemm_inner or traces or solver or sharded or fused" \
        tests/test_ops_gpu.py tests/test_traces_gpu.py tests/test_solver_gpu.py tests/test_distributed_gpu.py tests/test_fused_passes_gpu.py tests/test_exact_gpu.py || exit $?
      ;;
    selprobe)
      rm -rf "$OUT/selprof"
      step selprobe 300 rocprofv3 --kernel-trace --stats -d "$OUT/selprof" -o run --output-format csv -- \
        python3 tools/select_probe.py 12.5e6 --nsel 8,16 || exit $?
      ;;
    csab)
      for v in 0 1 0 1; do
        SSP_INNER_CS=$v SSP_LEDGER_DETAIL=1 step "csab_$v" 300 python -u tools/solver_ledger.py --configs C4-shard \
          --out "$OUT/c4_ledger_cs$v.json" || exit $?
      done
      ;;
    outercu)
      for v in 8 2 4 8 2 4; do
        SSP_OUTER_WG_PER_CU=$v step "outercu_$v" 300 python -u tools/size_probe.py --ops gemm_outer_set,gemm_outer,axpy_pairs_norm \
          --ns 6250000,12500000,25000000,100000000 --out "$OUT/outercu_$v.json" || exit $?
      done
      ;;
    outerab)
      step outerab 400 python -u tools/outer_cu_ab.py --out "$OUT/outer_cu_ab.json" || exit $?
      ;;
    selab)
      step selab 300 python -u tools/select_ab.py --out "$OUT/select_ab.json" || exit $?
      ;;
    selsizes)
      for n in 1.5e5 1.25e6 1.25e7 1e8; do
        step "selsize_$n" 200 python -u tools/select_probe.py $n --nsel 8,16 || exit $?
      done
      ;;
    kernargab)
      for round in 1 2; do
        step "ka_default_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag default || exit $?
        HIP_FORCE_DEV_KERNARG=1 step "ka_dev_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag dev_kernarg || exit $?
        HIP_FORCE_DEV_KERNARG=0 step "ka_host_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag host_kernarg || exit $?
        HSA_KERNARG_POOL_SIZE=33554432 step "ka_pool_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag pool32m || exit $?
      done
      ;;
    kernargab2)
      for round in 1 2 3; do
        step "kb_default_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag default || exit $?
        HIP_FORCE_DEV_KERNARG=1 step "kb_dev_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag dev_kernarg || exit $?
        HSA_KERNARG_POOL_SIZE=33554432 step "kb_pool_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag pool32m || exit $?
        HIP_FORCE_DEV_KERNARG=1 HSA_KERNARG_POOL_SIZE=33554432 step "kb_both_$round" 120 python -u tools/trace_c4.py --repeat 6 --tag both || exit $?
      done
      ;;
    fusedab)
      step fusedab 400 python -u tools/fused_cu_ab.py --out "$OUT/fused_cu_ab.json" || exit $?
      ;;
    gputests)
      step gputests 1500 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests || exit $?
      ;;
    shapetab)
      rm -rf "$OUT/shapetab"
      SSP_LEDGER_DETAIL=1 SSP_LEDGER_TIMING=dispatch step shapetab 300 rocprofv3 --kernel-trace -d "$OUT/shapetab" -o run \
        --output-format csv -- python3 tools/solver_ledger.py --configs C4-shard --out "$OUT/shapetab_ledger.json" || exit $?
      python3 tools/shape_table.py "$OUT/shapetab_ledger.json" "$OUT/shapetab/run_kernel_trace.csv" > "$OUT/shape_table.md" || exit $?
      ;;
    benchprof)
      rm -rf "$OUT/benchprof"
      step benchprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/benchprof" -o run --output-format csv -- \
        python3 -u bench.py --steps 10 --warmup 3 || exit $?
      grep '^{' "$OUT/benchprof.log" > "$OUT/bench_under_rocprof.json" || true
      ;;
    pmcbench)
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf "$OUT/pmcb_$c"
        step "pmcb_$c" 600 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmcb_$c" -o run --output-format csv -- \
          python3 bench.py --steps 2 --warmup 1 --ledger-steps 1 --no-cpu-baseline --no-in-solver --no-small || exit $?
      done
      ;;
    pmcc4)
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf "$OUT/pmcc4_$c"
        step "pmcc4_$c" 300 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmcc4_$c" -o run --output-format csv -- \
          python3 tools/solver_ledger.py --configs C4-shard --out "$OUT/pmcc4_ledger_$c.json" || exit $?
      done
      ;;
    shapes)
      for n in 1e8 1e7; do
        step "shapes_$n" 300 python -u tools/shapes_bench.py --n $n --reps 10 --out "$OUT/shapes_n$n.json" || exit $?
      done
      ;;
    smoke)
      step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
      ;;
    mergeab)
      for round in 1 2 3; do
        for v in 0 1; do
          SSP_SYNTH_MERGE=$v step "mab_${v}_$round" 120 python -u tools/wall_ab.py --repeat 8 --tag "merge$v" || exit $?
          grep '^{' "$OUT/mab_${v}_$round.log" >> "$OUT/merge_ab.jsonl" || true
        done
      done
      ;;
    synthtests)
      step synthtests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "synth or trace or solver or sharded" \
        tests/test_ops_gpu.py tests/test_traces_gpu.py tests/test_solver_gpu.py tests/test_distributed_gpu.py || exit $?
      ;;
    transab)
      step transab 300 python -u tools/transform_ab.py --out "$OUT/transform_ab.json" || exit $?
      ;;
    selkern)
      rm -rf "$OUT/selkern"
      step selkern 300 rocprofv3 --kernel-trace --stats -d "$OUT/selkern" -o run --output-format csv -- \
        python3 tools/select_probe.py 1.25e7 --nsel 8,16 || exit $?
      ;;
    c4trace)
      rm -rf "$OUT/c4trace"
      step c4trace 300 rocprofv3 --kernel-trace -d "$OUT/c4trace" -o run --output-format csv -- \
        python3 tools/trace_c4.py || exit $?
      ;;
    c4hiptrace)
      rm -rf "$OUT/c4hiptrace"
      step c4hiptrace 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$OUT/c4hiptrace" -o run --output-format csv -- \
        python3 tools/trace_c4.py || exit $?
      ;;
    gapprobe)
      step gapprobe 300 python -u tools/gap_probe.py --out "$OUT/gap_probe.json" || exit $?
      ;;
    sizeprobe)
      step sizeprobe 400 python -u tools/size_probe.py --out "$OUT/size_probe.json" || exit $?
      ;;
    c4prof)
      rm -rf "$OUT/c4prof"
      step c4prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4prof" -o run --output-format csv -- \
        python3 tools/solver_ledger.py --configs C4-shard --out "$OUT/c4prof_ledger.json" || exit $?
      ;;
    *)
      echo "unknown step $s"
      exit 2
      ;;
  esac
done
echo "session done"
