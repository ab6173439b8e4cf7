#!/bin/bash
# Round 5: tools/volume_probe.py's Decimate access shapes (units per wave,
# columns per lane, unit order, load policy) at 256, 512 and 1024 planes:
# does the 1024-plane launch's slowdown follow the access shape or the size?
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_vdecprobe; mkdir -p $OUT
export TMPDIR=/tmp
for z in 256 512 1024; do
  echo "== planes $z" | tee -a $OUT/probe.log
  timeout -k 10 300 python tools/volume_probe.py --planes $z --reps 20 >> $OUT/probe.log 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
echo "== done"
