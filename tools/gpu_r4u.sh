#!/bin/bash
# Round-4 GPU session U: the sparse op tests (publish-tail shapes), then the multi-process distributed suite, verbose, with durations (the
# full-size 8-shard C4 / C5 tests over peer memory included).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4u
mkdir -p "$OUT"
export TMPDIR=/tmp
(while sleep 60; do date +%T >> "$OUT/heartbeat"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "sparse" -m gpu -v -x --timeout 120 --timeout-method thread \
  > "$OUT/sparse.log" 2>&1 || { rc=$?; echo "sparse rc=$rc"; tail -20 "$OUT/sparse.log"; exit $rc; }
tail -2 "$OUT/sparse.log"
timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread \
  -rf --durations=10 > "$OUT/dist.log" 2>&1
rc=$?
echo "dist rc=$rc"; tail -14 "$OUT/dist.log"
exit $rc
