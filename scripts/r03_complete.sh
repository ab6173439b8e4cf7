#!/bin/bash
# Round 3: misaligned bands in burst-completion mode (no barrier) against the
# round-2 launch shapes; full GPU suite first.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_complete; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 3000x3000 2600x2600 2000x2000 1500x1500 1000x1000 2040x2048; do
    b "$sh" "X=0" --shape $sh
    b "$sh" "AQZ_BAND_COMPLETE=0" --shape $sh
    b "$sh" "AQZ_BAND_COMPLETE=0 AQZ_CASCADE_WAVES=6" --shape $sh
  done
  b "3000x3000_tiled" "X=0" --shape 3000x3000 --tiled
  b "f32_3000" "X=0" --shape 3000x3000 --workload 4096x4096_f32
  b "f32_3000" "AQZ_BAND_COMPLETE=0" --shape 3000x3000 --workload 4096x4096_f32
  b headline "X=0"
done
echo "== done"
