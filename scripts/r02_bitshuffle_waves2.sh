#!/bin/bash
# Bit shuffle with the word transpose: workgroup size A/B ($AQZ_BITSHUFFLE_WAVES).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/bswaves; mkdir -p $OUT
for rep in 1 2; do for wv in 1 2 4; do
  echo "waves=$wv" >> $OUT/bitshuffle_ts.log
  AQZ_BITSHUFFLE_WAVES=$wv timeout -k 10 200 python tools/bitshuffle_ts.py >> $OUT/bitshuffle_ts.log 2>&1 || { tail -20 $OUT/bitshuffle_ts.log; exit 1; }
done; done
grep -v amdgpu.ids $OUT/bitshuffle_ts.log
echo "== done"
