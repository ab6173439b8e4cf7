#!/bin/bash
# The zero-fill rule as shipped (rows cap for 1-byte types only): default
# lines on u8 and u16 camera frames, then the GPU suite and smoke.
set -e
out=gpurun_out/r04_zrows_confirm
mkdir -p $out
: > $out/ab.log
run() {  # workload shape
  timeout -k 10 120 python bench.py --workload $1 --shape $2 --tiled \
    --steps 20 --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);print('$1 $2 default', d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $out/ab.log
}
for shape in 2600x2600 2304x2304 3000x3000 5000x4000 512x512; do run 512x512_u8 $shape; done
for shape in 3000x3000 5472x3648 6000x4000 2600x2600 2000x2000 4096x4096; do run 4096x4096_u16 $shape; done
for shape in 3000x3000 6000x4000; do run 4096x4096_f32 $shape; done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $out/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
