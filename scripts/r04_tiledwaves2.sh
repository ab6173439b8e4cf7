#!/bin/bash
# Chunk-tiled cascade: waves per workgroup ($AQZ_TILED_WAVES) over frame
# widths of 4-14 column tiles, u16 and f32 (one round; same box).
set -e
out=gpurun_out/r04_tiledwaves2
mkdir -p $out
: > $out/ab.log
run() {  # workload shape waves
  AQZ_TILED_WAVES=$3 timeout -k 10 120 python bench.py --workload $1 --shape $2 --tiled --steps 20 \
    --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$1 $2 waves=$3', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
}
for shape in 2000x2000 2304x2304 3500x3500 4100x4100 4600x3000 7000x5000 2048x2048 3072x3072; do
  for w in 4 2 1 3; do run 4096x4096_u16 $shape $w; done
done
for shape in 3000x3000 6000x4000 5472x3648 2000x2000; do
  for w in 4 2; do run 4096x4096_f32 $shape $w; done
done
