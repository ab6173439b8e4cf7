#!/bin/bash
# Round 3: aligned 8-tile bands in 4-tile segments (2-3 workgroups per CU for
# 4096 f32 instead of one): parity with the knob on, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_seg4; mkdir -p $OUT
AQZ_BAND_SEG4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch or headline" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for m in max mean min decimate; do
    b "f32_$m" "X=0" --workload 4096x4096_f32 --method $m
    b "f32_$m" "AQZ_BAND_SEG4=1" --workload 4096x4096_f32 --method $m
  done
  b headline "X=0"
  b headline "AQZ_BAND_SEG4=1"
  b 3072 "X=0" --shape 3072x3072
  b 3072 "AQZ_BAND_SEG4=1" --shape 3072x3072
done
echo "== done"
