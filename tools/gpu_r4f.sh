#!/bin/bash
# Round-4 GPU session F: sharded short solves against the reference's MPI build (bit for bit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4f
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
step mpi_exact 600 python -u -m pytest tests/test_distributed_gpu.py -k "reference_mpi_build" -v -s --timeout 300 --timeout-method thread || exit $?
echo "session done"
