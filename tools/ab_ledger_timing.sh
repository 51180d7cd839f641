#!/bin/bash
# A/B of the ledger's timing (SSP_LEDGER_TIMING=events | dispatch) and of the synthetic apply's shape
# (SSP_SYNTH_SHAPE=window) on the C4 shard and C3, alternating processes, plus one kernel trace of the
# C4-shard solve (development tool).  Outputs under gpurun_out/ab_ledger/.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_ledger
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- \
  python3 tools/solver_ledger.py --configs C4-shard --out "$OUT/prof_c4_ledger.json" > "$OUT/prof_c4.log" 2>&1 || exit $?
echo "trace done"
for round in 1 2; do
  for v in events dispatch dispatch_window; do
    case $v in
      events) env_t=events; env_s= ;;
      dispatch) env_t=dispatch; env_s= ;;
      dispatch_window) env_t=dispatch; env_s=window ;;
    esac
    SSP_LEDGER_TIMING=$env_t SSP_SYNTH_SHAPE=$env_s timeout -k 10 200 python3 tools/solver_ledger.py \
      --configs C4-shard,C3 --out "$OUT/${v}_$round.json" > "$OUT/${v}_$round.log" 2>&1 || exit $?
    echo "$v round $round:"; grep -h '"config"' "$OUT/${v}_$round.log" | cut -c1-220
  done
done
