#!/bin/bash
# Round 4: misaligned >8-tile bands stored by their last two waves (new
# default) — parity, then u16 and f32 camera frames against one storing wave.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_last2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # tag workload shape env...
  local tag=$1 w=$2 sh=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --workload $w --shape $sh --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc \
    > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$tag', '$w', '$sh', r['avg_launch_us'], r['frac'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for w in 4096x4096_u16 4096x4096_f32; do
    for sh in 6000x4000 5472x3648 4100x4100; do
      b last1 $w $sh AQZ_BAND_LAST=1
      b default $w $sh
    done
  done
done
echo "== done"
