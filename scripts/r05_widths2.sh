#!/bin/bash
# Round 5: 16-byte tiles now the default for 4- and 8-byte types on
# line-aligned rows.  The whole GPU suite, then f64 / u32 Mean default lines
# and f64 chunk-tiled (default narrow vs AQZ_TILED_NARROW=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_widths2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {
  local label=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc $BARGS > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  BARGS="" run f64_mean_r$rep 4096x4096_f64 AQZ_UNUSED=0
  BARGS="" run u32_mean_r$rep 4096x4096_u32 AQZ_UNUSED=0
  BARGS="--tiled" run f64_tiled_narrow_r$rep 4096x4096_f64 AQZ_UNUSED=0
  BARGS="--tiled" run f64_tiled_wide_r$rep 4096x4096_f64 AQZ_TILED_NARROW=0
  BARGS="--tiled" run u32_tiled_narrow_r$rep 4096x4096_u32 AQZ_UNUSED=0
  BARGS="--tiled" run u32_tiled_wide_r$rep 4096x4096_u32 AQZ_TILED_NARROW=0
done
echo "== done"
