#!/bin/bash
# The CPU-path trace of C3 at full size with the rank-8 synthetic H (tests/golden/make_traces.py case
# C3_n1e8_rank8: the bench's own solve and C4's problem).  The CPU path holds ~96 GB per run, more
# than the build container has, so the runs go to a host with the memory (the GPU box's host; no GPU
# work): each given part (base / reordered / reordered_blocked) in its own process, in parallel, with
# the bit-identical OpenMP build of the oracle.  Outputs gpurun_out/c3r8_<part>.json, merged into
# tests/golden/traces.json with make_traces.py --merge.  Progress (elapsed, resident memory of each run)
# every 60 s.
# Usage: tools/trace_c3_n1e8.sh PART [PART]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
threads=$((16 / $#))
pids=()
for part in "$@"; do
  OMP_NUM_THREADS=$threads timeout -k 10 1100 python -u tests/golden/make_traces.py --omp --only C3_n1e8_rank8 \
    --part "$part" --out "$OUT/c3r8_$part.json" >"$OUT/c3r8_$part.log" 2>&1 &
  pids+=($!)
done
start=$(date +%s)
while :; do
  alive=0
  line="t=$(($(date +%s) - start))s"
  for p in "${pids[@]}"; do
    if kill -0 "$p" 2>/dev/null; then
      alive=1
      for c in $(pgrep -P "$p"); do line="$line rss[$c]=$(awk '/VmRSS/{printf "%.1fGB", $2/1e6}' /proc/$c/status 2>/dev/null)"; done
    fi
  done
  [ $alive = 0 ] && break
  echo "$line" | tee -a "$OUT/c3r8_progress.txt"
  sleep 60
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
cat "$OUT"/c3r8_*.log
exit $rc
