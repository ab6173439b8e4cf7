#!/bin/bash
# Round 5: 16-byte f32 tiles with the misaligned-segment store scheme, forced
# (AQZ_CASCADE_NARROW=1), against the default 32-byte tiles on camera widths
# whose rows split lines; the fuzz and parity suites under the forced tile
# first (test_take_frame_tiled left out: it counts the streaming path's
# one-launch tiled runs, which need the row-major and tiled tiles to agree,
# and forcing one side breaks that on purpose).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_misnarrow; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_CASCADE_NARROW=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_digests.py \
  -k "not take_frame_tiled" > $OUT/pytest_forced.log 2>&1 || { tail -40 $OUT/pytest_forced.log; exit 1; }
tail -1 $OUT/pytest_forced.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload 4096x4096_f32 --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc $BARGS > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for sh in 5472x3648 6000x4000 4100x4100 3000x3000 2000x2000; do
    BARGS="--shape $sh" run rm_${sh}_wide_r$rep AQZ_UNUSED=0
    BARGS="--shape $sh" run rm_${sh}_narrow_r$rep AQZ_CASCADE_NARROW=1
  done
done
echo "== done"
