#!/bin/bash
# Chunk-tiled zero fill: waves sized by overhang rows as well as bytes
# ($AQZ_TILED_ZROWS_PER_WAVE 32 = new default, 0 = the byte rule alone, 8),
# then the GPU suite on the new default.
set -e
out=gpurun_out/r04_zrows
mkdir -p $out
: > $out/ab.log
run() {  # workload shape zi
  AQZ_TILED_ZROWS_PER_WAVE=$3 timeout -k 10 120 python bench.py --workload $1 --shape $2 --tiled \
    --steps 20 --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$1 $2 zrows=$3', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
}
for shape in 2600x2600 2304x2304 1500x1500 3000x3000 5000x4000 4096x4096 512x512 2048x2048; do
  for z in 32 0 8; do run 512x512_u8 $shape $z; done
done
for round in 1 2; do
  for shape in 3000x3000 5472x3648 6000x4000 4096x4096 2304x2304; do
    for z in 32 0; do run 4096x4096_u16 $shape $z; done
  done
  for z in 32 0; do run 4096x4096_f32 3000x3000 $z; done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $out/pytest_gpu.log 2>&1
