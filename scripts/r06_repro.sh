#!/bin/bash
# Round 6: the reduced repro of DESIGN.md §12.1 (tools/divergent/repro.hip),
# divergent vs wave-uniform NaN branch, with and without forced-zero waits.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_repro; mkdir -p $OUT
for v in uni div uniwz divwz; do
  timeout -k 10 120 tools/divergent/repro_$v 200 > $OUT/$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; cat $OUT/$v.log
  [ $rc -eq 0 ] || exit $rc
done
echo "== done"
