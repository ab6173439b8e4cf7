#!/bin/bash
# Misaligned 5-8-tile bands: staging forced ($AQZ_BAND_FORCE level mask) now
# that the band kernel follows the load cache policy, vs direct stores and the
# tiled kernel.  r02t/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02t; mkdir -p $OUT
for i in 1 2; do
  for w in "--shape 3000x3000" "--shape 2600x2600" "--shape 4000x3000"; do
    for e in "X=0" "AQZ_BAND_FORCE=15" "AQZ_BAND_FORCE=1" "AQZ_BAND_FORCE=15 AQZ_LOAD_NT=1" "TILED=1"; do
      extra=""; [ "$e" = "TILED=1" ] && extra="--tiled"
      env $e timeout -k 10 120 python bench.py $w $extra --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$w', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/misal_ab.log
    done
  done
done
