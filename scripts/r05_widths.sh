#!/bin/bash
# Round 5: the 16-byte tile for the other 4-byte type (u32, on by default
# with f32) and for f64 (off by default), against the 32-byte tile, at
# 4096^2, Mean and Max, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_widths; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local label=$1 w=$2 m=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --workload $w --method $m --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for w in 4096x4096_u32 4096x4096_f64; do
    for m in mean max; do
      run ${w}_${m}_narrow_r$rep $w $m AQZ_CASCADE_NARROW=1
      run ${w}_${m}_wide_r$rep $w $m AQZ_CASCADE_NARROW=0
    done
  done
done
echo "== done"
