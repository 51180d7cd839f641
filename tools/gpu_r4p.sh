#!/bin/bash
# Round-4 GPU session P: HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) against the default,
# on the per-reduction latency and the C4-shard solve, alternating processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4p
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-240; if [ $rc -gt 1 ]; then return $rc; fi; return 0; }
for rep in 1 2; do
  step "lat_default_$rep" 300 python -u tools/latency_probe.py --out "$OUT/lat_default_$rep.json" || exit $?
  HIP_FORCE_DEV_KERNARG=1 step "lat_devkernarg_$rep" 300 python -u tools/latency_probe.py --out "$OUT/lat_devkernarg_$rep.json" || exit $?
  step "ab_default_$rep" 300 python -u tools/transport_ab.py --config C4-shard --reps 5 --out "$OUT/ab_default_$rep.json" || exit $?
  HIP_FORCE_DEV_KERNARG=1 step "ab_devkernarg_$rep" 300 python -u tools/transport_ab.py --config C4-shard --reps 5 --out "$OUT/ab_devkernarg_$rep.json" || exit $?
done
echo "session done"
