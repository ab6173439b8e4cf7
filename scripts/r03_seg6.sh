#!/bin/bash
# Round 3: aligned 5-7-tile bands (3072^2: 6, 2560x2160: 5, 3584^2: 7) in
# 3-tile segments (AQZ_BAND_SEG4=1 AQZ_BAND_SEGN=3) against whole bands.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_seg6; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_BAND_SEG4=1 AQZ_BAND_SEGN=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 3072x3072 2560x2160 3584x3584; do
    b u16_$sh "X=0" --shape $sh
    b u16_$sh "AQZ_BAND_SEG4=1 AQZ_BAND_SEGN=3" --shape $sh
  done
done
echo "== done"
