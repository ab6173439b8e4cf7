#!/bin/bash
# Round 3: band workgroups whose last wave stores the band (no barrier,
# $AQZ_BAND_LAST=1): parity with the knob on (and with every level of
# misaligned 5-8-tile bands staged), then A/B against the barrier form and
# against direct stores.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_last; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_BAND_LAST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch or headline" --timeout 120 --timeout-method thread > $OUT/pytest_last.log 2>&1 || { tail -30 $OUT/pytest_last.log; exit 1; }
tail -1 $OUT/pytest_last.log
AQZ_BAND_LAST=1 AQZ_BAND_FORCE=15 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch" --timeout 120 --timeout-method thread > $OUT/pytest_last_force.log 2>&1 || { tail -30 $OUT/pytest_last_force.log; exit 1; }
tail -1 $OUT/pytest_last_force.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  b headline "X=0"
  b headline "AQZ_BAND_LAST=1"
  b f32_mean "X=0" --workload 4096x4096_f32
  b f32_mean "AQZ_BAND_LAST=1" --workload 4096x4096_f32
  b 2000 "X=0" --shape 2000x2000
  b 2000 "AQZ_BAND_LAST=1" --shape 2000x2000
  for sh in 3000x3000 2600x2600 4000x3000; do
    b $sh "X=0" --shape $sh
    b $sh "AQZ_BAND_FORCE=15" --shape $sh
    b $sh "AQZ_BAND_FORCE=15 AQZ_BAND_LAST=1" --shape $sh
  done
done
echo "== done"
