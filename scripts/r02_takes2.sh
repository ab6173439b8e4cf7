#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/takes2; mkdir -p $OUT
for m in "" behind ondemand plain; do
  timeout -k 10 300 python tools/e2e_takes.py ${m:+--only $m} > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
  echo "-- only=${m:-all}"; grep ms/frame $OUT/t.log
done
echo "== done"
