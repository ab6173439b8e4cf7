#!/bin/bash
# Round 3: tiles per segment for aligned 8-tile bands, 3 against 4, over the
# methods and types the headline-width frames take (two rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_segn2; mkdir -p $OUT
export TMPDIR=/tmp
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for n in 4 3; do
    b headline "AQZ_BAND_SEGN=$n"
    b u16_min "AQZ_BAND_SEGN=$n" --method min
    b u16_max "AQZ_BAND_SEGN=$n" --method max
    b u16_decimate "AQZ_BAND_SEGN=$n" --method decimate
    b f32_max "AQZ_BAND_SEGN=$n" --workload 4096x4096_f32 --method max
    b u16_4096x2160 "AQZ_BAND_SEGN=$n" --shape 4096x2160
  done
done
echo "== done"
