#!/bin/bash
# Round 6 (rerun with the round-6 node APIs in the driver): the host-instrumented node driver (built here by
# scripts/sanitize_gpu_build.sh; its device code carries no sanitizer) on the
# GPU.  (1) ASan + UBSan, every case once, as the gate; (2) LeakSanitizer at
# 1 and 4 rounds of every case: the runtimes' one-off allocations stay the
# same, a leak in the library would grow with the rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_sanitize; mkdir -p $OUT
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 \
  timeout -k 10 300 tests/sanitize/bin/node_gpu > $OUT/node_gpu.log 2>&1 || { tail -40 $OUT/node_gpu.log; exit 1; }
cat $OUT/node_gpu.log
for r in 1 4; do
  ASAN_OPTIONS=detect_leaks=1:protect_shadow_gap=0 LSAN_OPTIONS=suppressions=$PWD/tests/sanitize/lsan.supp \
  AQZ_SAN_REPEAT=$r timeout -k 10 300 tests/sanitize/bin/node_gpu > $OUT/leaks_r$r.log 2>&1
  echo "rounds=$r exit=$? $(grep -c ' ok (' $OUT/leaks_r$r.log) cases ok; $(grep SUMMARY $OUT/leaks_r$r.log || echo 'no leaks')"
done
