#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_narrow_dbg2; mkdir -p $OUT
timeout -k 10 300 python tools/narrow_dbg.py > $OUT/dbg.log 2>&1; rc=$?
tail -80 $OUT/dbg.log
exit $rc
