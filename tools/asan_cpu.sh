#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU suite: the product's host
# layer and C API (iterative-solver_amd/host/*.cpp, include/itsolv_hbm/*.h, compiled into
# oracle/build/libitsolv_emul.so over the host emulation of the device ABI), oracle/ssp_emul.cpp, the
# oracle itself and the C++ component tests are built with -fsanitize=address,undefined; the Fortran
# test callers link against those libraries.  The sanitizer runtime is preloaded into the Python test
# process (python itself is not instrumented; leak checking is off for that reason).  Any report
# fails the run (halt_on_error).  Host code only: no GPU code is built or run here.
# Usage: tools/asan_cpu.sh [pytest args...]      (log: profiles/r3/asan_cpu.log)
set -u
cd "$(dirname "$0")/.."
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
LOG=${ASAN_LOG:-profiles/r3/asan_cpu.log}
mkdir -p "$(dirname "$LOG")"
make -B -j8 -C oracle SAN_FLAGS="$SAN" >/dev/null || exit 1
if [ -x /opt/rocm/bin/amdflang ]; then make -B -j8 -C tests/fortran >/dev/null || exit 1; fi
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
{
  echo "# tools/asan_cpu.sh $(date -u +%FT%TZ)  SAN_FLAGS=$SAN"
  LD_PRELOAD="$PRE" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 ITSOLV_SAN_FLAGS="$SAN" \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
} >"$LOG" 2>&1
rc=$?
grep -n "ERROR: AddressSanitizer\|runtime error:" "$LOG" | head -20
tail -n 3 "$LOG"
# back to the regular (uninstrumented) build
make -B -j8 -C oracle >/dev/null && { [ ! -x /opt/rocm/bin/amdflang ] || make -B -j8 -C tests/fortran >/dev/null; }
exit $rc
