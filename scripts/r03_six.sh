#!/bin/bash
# Round 3: 6-tile u16 bands (3000^2, 2600^2): last-wave staging (default)
# against direct stores (AQZ_BAND_MIS_MAX=4), two rounds, with and without
# the PMC child run the closing script adds.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_six; mkdir -p $OUT
export TMPDIR=/tmp
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 3000x3000 2600x2600 2304x2304; do
    b u16_$sh "X=0" --shape $sh --no-pmc
    b u16_$sh "AQZ_BAND_MIS_MAX=4" --shape $sh --no-pmc
  done
  b u16_3000x3000_pmc "X=0" --shape 3000x3000
  b headline "X=0" --no-pmc
done
echo "== done"
