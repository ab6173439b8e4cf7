#!/bin/bash
# Round 5: small-unit chunk-tiled cascades now load plain.  Tiled, lattice,
# fuzz and parity suites, then the default against AQZ_LOAD_NT=1, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_tilednt2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_tiled.py tests/test_gpu_lattice.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_adapter.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {
  local label=$1 w=$2 m=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --workload $w --method $m --tiled --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for wm in 512x512_u8:decimate 512x512_u8:mean 2048x2048_u16:decimate 4096x4096_u16:mean; do
    w=${wm%%:*}; m=${wm##*:}
    run t_${w}_${m}_default_r$rep $w $m AQZ_UNUSED=0
    run t_${w}_${m}_nt_r$rep $w $m AQZ_LOAD_NT=1
  done
done
echo "== done"
