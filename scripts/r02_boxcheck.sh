#!/bin/bash
# Box check: headline with direct stores vs staged 8-wave bands, and the
# tiled kernel, alternating twice (about 40 s).  Appends to gpurun_out/r02s/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02s; mkdir -p $OUT
tag=$(date +%H%M%S)
for i in 1 2; do
  for e in "AQZ_BAND_ALIGNED=0" "X=0" "TILED=1"; do
    extra=""; [ "$e" = "TILED=1" ] && extra="--tiled"
    env $e timeout -k 10 120 python bench.py $extra --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check > $OUT/ab_$tag.json 2> $OUT/ab_$tag.err || { tail -5 $OUT/ab_$tag.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_$tag.json'));r=d['roofline'];print('$tag', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'])" | tee -a $OUT/boxcheck_$tag.log
  done
done
