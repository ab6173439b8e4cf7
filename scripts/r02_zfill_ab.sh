#!/bin/bash
# Tiled cascade: what the zero-fill waves cost on shapes whose tiles overhang
# the levels ($AQZ_TILED_ZWAVES: default, 0 = skipped, or a count), two
# alternating passes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/zfill; mkdir -p $OUT
for pass in 1 2; do
  for s in 3000x3000 5472x3648 2000x2000 3072x3072 4096x4096; do
    for zw in "" 0 1024 256; do
      AQZ_TILED_ZWAVES=$zw timeout -k 10 200 python bench.py --shape $s --tiled --no-check --cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 20 --warmup 5 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/k.json'));r=d['roofline'];print('pass $pass','$s','zw=${zw:-default}',r['avg_launch_us'],r['achieved'],r['frac'])" | tee -a $OUT/zfill_ab.txt
    done
  done
done
echo "== done"
