#!/bin/bash
# Round 3: misaligned segments on by default for bands of more than 8 tiles
# (2- and 4-byte types).  Full GPU suite, then default against
# AQZ_BAND_MIS_SEG=0 (band workgroups, direct stores).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_misseg_confirm; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for e in "X=0" "AQZ_BAND_MIS_SEG=0"; do
    b f32_5472x3648 "$e" --workload 4096x4096_f32 --shape 5472x3648
    b u16_6000x4000 "$e" --shape 6000x4000
    b u16_5472x3648 "$e" --shape 5472x3648
  done
  b u16_4000x3000 "X=0" --shape 4000x3000
  b headline "X=0"
  b f32 "X=0" --workload 4096x4096_f32
done
echo "== done"
