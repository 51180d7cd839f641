#!/bin/bash
# A/B of the fused-Gram transform's grid (SSP_GRAM_WG_PER_CU: default = its occupancy, or 8) in the
# microbenchmark and in the C4-shard / C3 solves, alternating processes (development tool).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_gram
mkdir -p "$OUT"
for round in 1 2; do
  for v in occ 8; do
    if [ $v = occ ]; then unset SSP_GRAM_WG_PER_CU; else export SSP_GRAM_WG_PER_CU=$v; fi
    timeout -k 5 120 tools/mb_transform_lib 10 > "$OUT/mb_${v}_$round.txt" 2>&1 || exit $?
    echo "mb $v round $round:"; grep -E "transform_gram" "$OUT/mb_${v}_$round.txt"
    timeout -k 10 200 python3 tools/solver_ledger.py --configs C4-shard,C3 --out "$OUT/ledger_${v}_$round.json" \
      > "$OUT/ledger_${v}_$round.log" 2>&1 || exit $?
    python3 -c "
import json,sys
for e in json.load(open('$OUT/ledger_${v}_$round.json')):
    o=e['ops'].get('transform_gram',{})
    print(e['config'], 'wall', e['wall_s'], 'kernel_ms', e['kernel_ms'], 'transform_gram_ms', o.get('ms'), o.get('GBs'))
"
  done
done
