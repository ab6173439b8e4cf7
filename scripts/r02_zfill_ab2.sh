#!/bin/bash
# Tiled cascade zero fill: count of zero-fill waves and their place in the
# grid ($AQZ_TILED_ZWAVES, $AQZ_TILED_ZLAST=1: after the cascade blocks),
# two alternating passes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/zfill2; mkdir -p $OUT
run() { # label env... -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --tiled --cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 20 --warmup 5 $ARGS > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/k.json'));r=d['roofline'];print('pass $pass','$ARGS','$label',r['avg_launch_us'],r['achieved'],r['frac'],d['config']['check'])" | tee -a $OUT/zfill_ab2.txt
}
for pass in 1 2; do
  for ARGS in "--shape 3000x3000" "--shape 5472x3648" "--shape 3072x3072" "--shape 2000x2000" "--workload 512x512_u8" "--workload 2048x2048_u16" "--workload 4096x4096_f32"; do
    run first4096 AQZ_TILED_ZLAST=0
    run first512 AQZ_TILED_ZLAST=0 AQZ_TILED_ZWAVES=512
    run first256 AQZ_TILED_ZLAST=0 AQZ_TILED_ZWAVES=256
    run last4096 AQZ_TILED_ZLAST=1
    run last1024 AQZ_TILED_ZLAST=1 AQZ_TILED_ZWAVES=1024
    run last256 AQZ_TILED_ZLAST=1 AQZ_TILED_ZWAVES=256
  done
done
echo "== done"
