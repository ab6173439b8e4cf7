#!/bin/bash
# Round 5: 16-byte tiles are now the f32 default.  The whole GPU suite, then
# f32 camera shapes row-major (default narrow vs AQZ_CASCADE_NARROW=0) and
# chunk-tiled (default narrow vs AQZ_TILED_NARROW=0), twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_narrow2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload 4096x4096_f32 --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc $BARGS > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for sh in 5472x3648 6000x4000 2000x2000 4096x4096; do
    BARGS="--shape $sh" run rm_${sh}_narrow_r$rep AQZ_UNUSED=0
    BARGS="--shape $sh" run rm_${sh}_wide_r$rep AQZ_CASCADE_NARROW=0
    BARGS="--shape $sh --tiled" run t_${sh}_narrow_r$rep AQZ_UNUSED=0
    BARGS="--shape $sh --tiled" run t_${sh}_wide_r$rep AQZ_TILED_NARROW=0
  done
done
echo "== done"
