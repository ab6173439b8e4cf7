#!/bin/bash
# Round 4: whole misaligned bands of 9-16 tiles in one workgroup of up to
# 1024 threads ($AQZ_BAND_WIDE=K: stored by the last K waves) — parity with
# K=2 (batch + fuzz), then A/B against the default 4-tile segments.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_wide; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_BAND_WIDE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "batch or fuzz" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
b() { # tag shape env...
  local tag=$1 sh=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --shape $sh --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 \
    > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];t=r.get('traffic_detail') or {}
print('$tag', '$sh', r['avg_launch_us'], r['frac'], t.get('write_bytes') and round(t['write_bytes']/(r['alg_bytes_per_launch']-r['alg_read_bytes_per_launch']),4), d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 6000x4000 5472x3648 4600x3000; do
    b default $sh
    b wide1 $sh AQZ_BAND_WIDE=1
    b wide2 $sh AQZ_BAND_WIDE=2
    b wide4 $sh AQZ_BAND_WIDE=4
  done
done
echo "== done"
