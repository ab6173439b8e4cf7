#!/bin/bash
# Round 6: the fuzz sweep widened from 256 to 4096 seeded cases (device
# batch, stream, tiled, Z stacks), once, on the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_fuzzwide; mkdir -p $OUT
AQZ_FUZZ_CASES=4096 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/fuzz4096.log 2>&1
rc=$?
tail -1 $OUT/fuzz4096.log
grep -h "AssertionError: case" $OUT/fuzz4096.log | cut -c1-220 | head -20
echo "== done rc=$rc"
