#!/bin/bash
# The 2/4-wave rule against forced 4-wave blocks (the old launch), then the
# whole GPU suite on the new default.
set -e
out=gpurun_out/r04_tiledwaves_confirm
mkdir -p $out
: > $out/ab.log
run() {  # workload shape waves(0 = default)
  if [ "$3" = 0 ]; then e=""; else e="AQZ_TILED_WAVES=$3"; fi
  env $e timeout -k 10 120 python bench.py --workload $1 --shape $2 --tiled --steps 20 \
    --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);c=d['config'];print('$1 $2 waves=$3', d['roofline']['avg_launch_us'], d['roofline']['frac'], c['batch_path'], c['launches_per_step'])" >> $out/ab.log
}
for round in 1 2; do
  for shape in 3000x3000 2600x2600 5472x3648 6000x4000 2000x2000 4096x4096 7000x5000; do
    for w in 0 4; do run 4096x4096_u16 $shape $w; done
  done
  for shape in 3000x3000 6000x4000; do for w in 0 4; do run 4096x4096_f32 $shape $w; done; done
done
run 512x512_u8 2600x2600 0
run 512x512_u8 512x512 0
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $out/pytest_gpu.log 2>&1
