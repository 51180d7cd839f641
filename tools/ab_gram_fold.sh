#!/bin/bash
# A/B of the fused-Gram transform's dot reduction (development tool): SSP_GRAM_FOLD=kernel (the last
# workgroup folds, one resident round of workgroups) against the default reduce pass after a full-grid
# kernel; solver ledgers of C4-shard and C3, alternating, two processes each.
set -e
out=${1:-gpurun_out/ab_gram_fold}
mkdir -p "$out"
for r in 1 2; do
  for v in kernel pass; do
    SSP_GRAM_FOLD=$v timeout -k 10 200 python -u tools/solver_ledger.py --configs C4-shard,C3 --out "$out/ledger_${v}_$r.json" > "$out/ledger_${v}_$r.log" 2>&1
    echo "$v $r done"
  done
done
