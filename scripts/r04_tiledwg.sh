#!/bin/bash
# Round 4: band-aligned workgroups for the chunk-tiled cascade on rows that
# split 128-B lines — parity (full suite), then A/B against 4-wave blocks
# ($AQZ_TILED_BAND_WG=0), two rounds, with PMC reads.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_tiledwg; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # tag workload shape env...
  local tag=$1 w=$2 sh=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --workload $w --shape $sh --tiled --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 \
    > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];t=r.get('traffic_detail') or {}
print('$tag', '$w', '$sh', r['avg_launch_us'], r['frac'], t.get('read_bytes') and round(t['read_bytes']/r['alg_read_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 3000x3000 2600x2600 5472x3648 2000x2000 6000x4000; do
    b wg0 4096x4096_u16 $sh AQZ_TILED_BAND_WG=0
    b wg1 4096x4096_u16 $sh
  done
  for sh in 3000x3000 6000x4000; do
    b wg0 4096x4096_f32 $sh AQZ_TILED_BAND_WG=0
    b wg1 4096x4096_f32 $sh
  done
done
echo "== done"
