#!/bin/bash
# Chunk-tiled cascade: waves per workgroup ($AQZ_TILED_WAVES) on camera
# frames and the headline, same box, two alternating rounds.
set -e
out=gpurun_out/r04_tiledwaves
mkdir -p $out
: > $out/ab.log
for round in 1 2; do
  for shape in 3000x3000 5472x3648 6000x4000 2600x2600 4096x4096; do
    for w in 4 2 8; do
      AQZ_TILED_WAVES=$w timeout -k 10 120 python bench.py --shape $shape --tiled --steps 20 \
        --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
      python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$round $shape waves=$w', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
    done
  done
done
