#!/bin/bash
# Chunk-tiled u8 frames (chunk 128): wide (1024-px) against half-width
# (512-px) column tiles ($AQZ_TILED_NARROW), same box, two rounds.
set -e
out=gpurun_out/r04_u8narrow
mkdir -p $out
: > $out/ab.log
run() {  # shape narrow
  AQZ_TILED_NARROW=$2 timeout -k 10 120 python bench.py --workload 512x512_u8 --shape $1 --tiled \
    --steps 20 --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$1 narrow=$2', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
}
for round in 1 2; do
  for shape in 2600x2600 3000x3000 2048x2048 6000x4000 5000x4000 512x512 4096x4096 2304x2304 1500x1500; do
    for n in 0 1; do run $shape $n; done
  done
done
