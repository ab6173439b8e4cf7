#!/bin/bash
# Round 3: tiles per segment for aligned 8-tile bands ($AQZ_BAND_SEGN, A/B;
# default 4): parity with 2 and 3, then 2 / 3 / 4 on the headline and F.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_segn; mkdir -p $OUT
export TMPDIR=/tmp
for n in 2 3; do
  AQZ_BAND_SEGN=$n timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -q -x -k "device_batch or headline or fuzz_device" --timeout 120 --timeout-method thread > $OUT/pytest_$n.log 2>&1 || { tail -30 $OUT/pytest_$n.log; exit 1; }
  tail -1 $OUT/pytest_$n.log
done
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for n in 4 2 3; do
    b headline "AQZ_BAND_SEGN=$n"
    b f32_mean "AQZ_BAND_SEGN=$n" --workload 4096x4096_f32
    b f32_min "AQZ_BAND_SEGN=$n" --workload 4096x4096_f32 --method min
    b f32_decimate "AQZ_BAND_SEGN=$n" --workload 4096x4096_f32 --method decimate
  done
done
echo "== done"
