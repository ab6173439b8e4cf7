#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
tail -1 $OUT/pytest_tiled.log 2>/dev/null
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check --steps 30 --warmup 5"
for rep in 1 2; do
for args in "--workload 512x512_u8 --tiled" "--workload 512x512_u8 --chunk 256 --tiled" "--tiled" "--workload 2048x2048_u16 --tiled"; do
  for r in 0 1; do
    AQZ_XCD_REMAP=$r timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { echo "FAIL $args"; tail -20 $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('remap=$r','$args'.ljust(44),d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))"
  done
done
done
