#!/bin/bash
# A/B of the XCD-contiguous block order ($AQZ_XCD_REMAP) on tiled and
# row-major cascades, alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check --steps 30 --warmup 5"
for rep in 1 2; do
for args in "" "--tiled" "--shape 5472x3648 --tiled" "--shape 3000x3000 --tiled" "--shape 3000x3000" "--shape 5472x3648"; do
  for r in 0 1; do
    AQZ_XCD_REMAP=$r timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('remap=$r','$args',d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))" | tee -a $OUT/remap_ab.log
  done
done
done
echo "== done"
