#!/bin/bash
# u8 chunk-tiled zero fill: rows per wave 32 (default), 16, 4 and 1.
set -e
out=gpurun_out/r04_zrows_u8
mkdir -p $out
: > $out/ab.log
run() {  # shape zi
  AQZ_TILED_ZROWS_PER_WAVE=$2 timeout -k 10 120 python bench.py --workload 512x512_u8 --shape $1 \
    --tiled --steps 20 --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$1 zrows=$2', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
}
for shape in 2600x2600 2304x2304 3000x3000 5000x4000 1500x1500 512x512; do
  for z in 32 16 4 1; do run $shape $z; done
done
