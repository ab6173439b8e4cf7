#!/bin/bash
# Chunk-tiled cascade on camera frames: load policy and XCD block order, as
# env A/B against the defaults (same box, two alternating rounds).
set -e
out=gpurun_out/r04_tiledknobs
mkdir -p $out
: > $out/ab.log
for round in 1 2; do
  for shape in 3000x3000 5472x3648 6000x4000 2600x2600; do
    for v in default nt1 remap1; do
      envs=""
      [ $v = nt1 ] && envs="AQZ_LOAD_NT=1"
      [ $v = remap1 ] && envs="AQZ_XCD_REMAP=1"
      env $envs timeout -k 10 120 python bench.py --shape $shape --tiled --steps 20 --warmup 3 \
        --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
      python -c "import json,sys;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$round $shape $v', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
    done
  done
done
