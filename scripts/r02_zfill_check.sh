#!/bin/bash
# Zero-fill waves sized by overhang bytes: tiled parity tests, then the new
# default against fixed counts (incl. big chunks, where the overhang exceeds
# the level data), two alternating passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/zfill3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiled.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_tiled.log 2>&1 || { tail -30 $OUT/pytest_tiled.log; exit 1; }
tail -1 $OUT/pytest_tiled.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --tiled --cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 20 --warmup 5 $ARGS > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/k.json'));r=d['roofline'];print('pass $pass','$ARGS','$label',r['avg_launch_us'],r['achieved'],r['frac'],d['config']['check'])" | tee -a $OUT/zfill_check.txt
}
for pass in 1 2; do
  for ARGS in "--shape 3000x3000" "--shape 5472x3648" "--shape 3072x3072" "--shape 2000x2000" "--workload 512x512_u8" "--shape 2000x2000 --chunk 1024" "--shape 3000x3000 --chunk 512"; do
    run bytes AQZ_X=0
    run w512 AQZ_TILED_ZWAVES=512
    run w4096 AQZ_TILED_ZWAVES=4096
  done
done
echo "== done"
