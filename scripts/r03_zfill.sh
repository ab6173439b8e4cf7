#!/bin/bash
# Round 3: what the tile overhang's zero fill costs on heavy-overhang shapes
# (AQZ_TILED_ZWAVES=0 leaves the overhang unwritten: A/B only), tiled batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_zfill; mkdir -p $OUT
export TMPDIR=/tmp
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['alg_bytes_per_launch'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 2304x2304 2600x2600 3000x3000 4096x4096; do
    b tiled_$sh "X=0" --tiled --shape $sh
    b tiled_$sh "AQZ_TILED_ZWAVES=0" --tiled --shape $sh
  done
done
echo "== done"
