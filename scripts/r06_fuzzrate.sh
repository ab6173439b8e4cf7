#!/bin/bash
# Round 6: how often does the row-local select form of the
# edge loads (lib_rowsel) give a wrong output, against the product (masked
# edge loads)?  The device-batch and stream fuzz, 30 times each, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_fuzzrate; mkdir -p $OUT
for rep in $(seq 1 30); do
  for v in product rowsel; do
    lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
    [ $v = rowsel ] && lib=$PWD/tools/divergent/lib_rowsel.so
    AQZ_LIB_PATH=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "device_batch or stream" > $OUT/fuzz_${v}_$rep.log 2>&1
    rc=$?
    echo "$v rep $rep rc=$rc $(tail -1 $OUT/fuzz_${v}_$rep.log)" | tee -a $OUT/summary.txt
    grep -h "AssertionError: case" $OUT/fuzz_${v}_$rep.log | cut -c1-220 | tee -a $OUT/summary.txt
    [ $rc -le 1 ] || exit $rc
  done
done
echo "== done"
