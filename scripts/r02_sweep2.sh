#!/bin/bash
# Round-2 closing sweep: every BASELINE config with the default bench line
# (PMC traffic, CPU baseline), the tiled headline, and the staged/direct band
# A/B on the headline (box check).  gpurun_out/r02l/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02l; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for e in "AQZ_BAND_ALIGNED=0" "X=0"; do
    env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'])" | tee -a $OUT/box_ab.log
  done
done
for w in 4096x4096_u16 4096x4096_f32 2048x2048_u16 512x512_u8 1024x1024x256_u16; do
  timeout -k 10 400 python bench.py --workload $w --cpu-seconds 5 > $OUT/sweep_$w.json 2> $OUT/sweep_$w.err || { tail -20 $OUT/sweep_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sweep_$w.json'));r=d['roofline'];print('$w',d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'),r['traffic'],d['config']['check'])"
done
timeout -k 10 300 python bench.py --tiled --cpu-seconds 0 --e2e-frames 0 > $OUT/bench_tiled.json 2> $OUT/bench_tiled.err || { tail -20 $OUT/bench_tiled.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_tiled.json'));r=d['roofline'];print('tiled',d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],r['traffic'])"
echo "== done"
