#!/bin/bash
# Pitch floor: the row-shaped HBM probe over each frame shape, then the
# kernel itself (row-major and chunk-tiled) on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/pitch; mkdir -p $OUT
echo "== probe"
timeout -k 10 300 python tools/pitch_probe.py --json $OUT/pitch_probe.jsonl > $OUT/pitch_probe.log 2>&1 || { tail -20 $OUT/pitch_probe.log; exit 1; }
cat $OUT/pitch_probe.log
echo "== kernel"
for s in 4096x4096 3000x3000 5472x3648 4100x4100 2000x2000; do
  for t in "" "--tiled"; do
    timeout -k 10 200 python bench.py --shape $s $t --cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 20 --warmup 5 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/k.json'));r=d['roofline'];print('$s','${t:-rowmajor}',r['avg_launch_us'],r['achieved'],r['frac'])" | tee -a $OUT/kernel.txt
  done
done
echo "== done"
