#!/bin/bash
# Round 5: small 1-byte pyramids chunk-tiled with 4 units per wave.  Tiled,
# lattice, fuzz, parity and adapter suites, then 512^2 u8 every method (the
# default against AQZ_TILED_UPW=0) and a 4-level u8 control, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_tiledupw; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_tiled.py tests/test_gpu_lattice.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_adapter.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
AQZ_TILED_UPW=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_tiled.py tests/test_gpu_lattice.py tests/test_gpu_fuzz.py -k "tiled or lattice" \
  > $OUT/pytest_forced.log 2>&1 || { tail -40 $OUT/pytest_forced.log; exit 1; }
tail -1 $OUT/pytest_forced.log
run() {
  local label=$1 m=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload 512x512_u8 --method $m --tiled --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc $BARGS > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for m in decimate mean min max; do
    BARGS="" run t512_${m}_default_r$rep $m AQZ_UNUSED=0
    BARGS="" run t512_${m}_upw1_r$rep $m AQZ_TILED_UPW=0
  done
done
echo "== done"
