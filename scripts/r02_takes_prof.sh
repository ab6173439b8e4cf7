#!/bin/bash
# Kernel and copy trace of the tiled-behind-the-pyramid takes against the
# on-demand ones (tools/e2e_takes.py), 16 frames each.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/takes_prof; mkdir -p $OUT
export TMPDIR=/tmp
for m in behind ondemand; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/$m -o run -- \
    python3 tools/e2e_takes.py --only $m --passes 1 --frames 16 > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
  grep "ms/frame" $OUT/$m.log
  for f in $(find $OUT/$m -name "*stats.csv"); do echo "-- $f"; head -12 $f | cut -c1-220; done
done
echo "== done"
