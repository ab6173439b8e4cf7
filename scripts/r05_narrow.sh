#!/bin/bash
# Round 5: f32 / f64 cascades with 16-byte tiles (AQZ_CASCADE_NARROW=1: 73
# VGPRs, 6 waves per SIMD) against the default 32-byte tiles (138 VGPRs, 3
# waves), every method, config F and two other f32 widths, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_narrow; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload 4096x4096_f32 --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc $BARGS > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for m in mean max decimate; do
    BARGS="--method $m" run f32_${m}_wide_r$rep AQZ_UNUSED=0
    BARGS="--method $m" run f32_${m}_narrow_r$rep AQZ_CASCADE_NARROW=1
  done
  for sh in 8192x2048 3072x3072; do
    BARGS="--shape $sh" run f32_${sh}_wide_r$rep AQZ_UNUSED=0
    BARGS="--shape $sh" run f32_${sh}_narrow_r$rep AQZ_CASCADE_NARROW=1
  done
done
echo "== done"
