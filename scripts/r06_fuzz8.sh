#!/bin/bash
# Round 6: the product's fuzz suite eight more times on one
# box (every variant: device batch, stream, tiled, Z stacks) — the masked
# edge loads' record under the default launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_fuzz8; mkdir -p $OUT
for rep in 1 2 3 4 5 6 7 8; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/fuzz_$rep.log 2>&1
  rc=$?
  echo "rep $rep rc=$rc $(tail -1 $OUT/fuzz_$rep.log)" | tee -a $OUT/summary.txt
  [ $rc -le 1 ] || exit $rc
done
echo "== done"
