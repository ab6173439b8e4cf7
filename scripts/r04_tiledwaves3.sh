#!/bin/bash
# Chunk-tiled cascade, waves per workgroup: the candidates of the two rules
# ("4 if the band's tile count divides by 4, else 2" and "the largest of
# 4/3/2/1 dividing it") where they differ, plus u8 and f64 (same box).
set -e
out=gpurun_out/r04_tiledwaves3
mkdir -p $out
: > $out/ab.log
run() {  # workload shape waves
  AQZ_TILED_WAVES=$3 timeout -k 10 120 python bench.py --workload $1 --shape $2 --tiled --steps 20 \
    --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$1 $2 waves=$3', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
}
for round in 1 2; do
  for shape in 3000x3000 2600x2600; do for w in 4 2 3; do run 4096x4096_u16 $shape $w; done; done
  for shape in 5472x3648 2304x2304; do for w in 4 2 1; do run 4096x4096_u16 $shape $w; done; done
  for w in 4 2 1; do run 4096x4096_f32 5472x3648 $w; done
  for shape in 3000x3000 6000x4000 5000x4000 2600x2600; do for w in 4 2 1; do run 512x512_u8 $shape $w; done; done
done
