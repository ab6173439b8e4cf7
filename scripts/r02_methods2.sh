#!/bin/bash
# Round-2 closing: every method on the headline and f32 configs with the
# final code (PMC traffic, CPU baseline), plus direct vs staged headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/r02p; mkdir -p $OUT
for e in "AQZ_BAND_ALIGNED=0" "X=0" "AQZ_BAND_ALIGNED=0" "X=0"; do
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'])" | tee -a $OUT/box_ab.log
done
for w in 4096x4096_u16 4096x4096_f32; do
  for m in decimate mean min max; do
    timeout -k 10 300 python bench.py --workload $w --method $m --cpu-seconds 3 --e2e-frames 0 > $OUT/${w}_$m.json 2> $OUT/${w}_$m.err || { tail -20 $OUT/${w}_$m.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${w}_$m.json'));r=d['roofline'];print('$w $m',d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],r['traffic'],r['alg_bytes_per_launch'],d['config']['check'])"
  done
done
echo "== done"
