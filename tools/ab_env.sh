#!/bin/bash
# A/B of an environment knob on the solver ledgers (development tool): for each value of VAR, two
# processes alternating, tools/solver_ledger.py on CONFIGS.
#   tools/ab_env.sh OUT_DIR VAR "v1 v2 ..." [CONFIGS]
set -e
out=$1; var=$2; vals=$3; configs=${4:-C4-shard}
mkdir -p "$out"
for r in 1 2; do
  for v in $vals; do
    env "$var=$v" timeout -k 10 200 python -u tools/solver_ledger.py --configs "$configs" --out "$out/ledger_${v}_$r.json" > "$out/ledger_${v}_$r.log" 2>&1
    echo "$var=$v rep $r done"
  done
done
