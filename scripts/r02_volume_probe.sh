#!/bin/bash
# Volume Decimate: the rows probe with the volume kernel's read patterns
# (every row of every plane / every other row of every other plane) beside
# the kernel itself at the same plane widths, same box, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/volprobe; mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 300 python tools/pitch_probe.py --set volume --json $OUT/probe_$rep.jsonl > $OUT/probe_$rep.log 2>&1 || { tail -20 $OUT/probe_$rep.log; exit 1; }
  grep -v amdgpu.ids $OUT/probe_$rep.log
  timeout -k 10 300 python tools/volume_shape_probe.py > $OUT/kernel_$rep.log 2>&1 || { tail -20 $OUT/kernel_$rep.log; exit 1; }
  grep -v amdgpu.ids $OUT/kernel_$rep.log
done
echo "== done"
