#!/bin/bash
# Round-3 A/B session (one GPU call): the gemm_inner row kernel's window vs stride shape
# (tools/row_shape_ab.py) and the reduction-result hand-off, k_publish kernel vs D2H copy + stream
# flag write (SSP_PUBLISH=copy), on the fused single-rank path and on a one-rank RCCL communicator
# (tools/latency_probe.py).  Each step has its own time limit; the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python tools/row_shape_ab.py --out "$OUT/row_shape_ab.json" || exit $?
for mode in kernel copy; do
  for comm in fused rccl; do
    flag=""
    [ "$comm" = rccl ] && flag="--rccl"
    echo "== publish=$mode comm=$comm"
    SSP_PUBLISH=$mode timeout -k 10 300 python tools/latency_probe.py $flag --out "$OUT/latency_${mode}_${comm}.json" || exit $?
  done
done
echo "ab session done"
