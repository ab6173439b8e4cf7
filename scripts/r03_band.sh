#!/bin/bash
# Round 3: vectorised LDS staging writes (f32 band bank conflicts) — full GPU
# suite, then f32 methods and the headline A/B against the 64 KiB cap, then
# the misaligned 3000^2 / 2600^2 / 5472x3648 shapes with one-band workgroups
# and write-back stores (env knobs only).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_band; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for m in max min decimate mean; do
    b "f32_$m" "X=0" --workload 4096x4096_f32 --method $m
    b "f32_$m" "AQZ_BAND_LDS_CAP=65536" --workload 4096x4096_f32 --method $m
  done
  b headline "X=0"
  b headline "AQZ_BAND_ALIGNED=0"
done
for i in 1 2; do
  for sh in 3000x3000 2600x2600 5472x3648; do
    b "$sh" "X=0" --shape $sh
    b "$sh" "AQZ_CASCADE_WAVES=6" --shape $sh
    b "$sh" "AQZ_CASCADE_WAVES=6 AQZ_STORE_WB=15" --shape $sh
    b "$sh" "AQZ_CASCADE_WAVES=8 AQZ_STORE_WB=15" --shape $sh
    b "$sh" "AQZ_STORE_WB=15" --shape $sh
  done
done
echo "== done"
