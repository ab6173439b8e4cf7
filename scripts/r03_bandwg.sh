#!/bin/bash
# Round 3: band-aligned direct workgroups for misaligned rows wider than 4
# tiles; parity first, then A/B against 4-wave blocks ($AQZ_BAND_WG=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_bandwg; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 3000x3000 2600x2600 5472x3648 4100x4100 4000x3000 2112x2048; do
    b "$sh" "X=0" --shape $sh
    b "$sh" "AQZ_BAND_WG=0" --shape $sh
  done
  b "f32_3000" "X=0" --shape 3000x3000 --workload 4096x4096_f32
  b "f32_3000" "AQZ_BAND_WG=0" --shape 3000x3000 --workload 4096x4096_f32
  b "3000_tiled" "X=0" --shape 3000x3000 --tiled
  b "5472_tiled" "X=0" --shape 5472x3648 --tiled
  b headline "X=0"
done
echo "== done"
