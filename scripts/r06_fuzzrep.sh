#!/bin/bash
# Round 6: the row-local select form of the edge loads gave
# one wrong pixel (fuzz case 181, u16) in one default fuzz run.  The device
# batch fuzz four times on each library: the product (exec-masked edge loads,
# as in round 5), lib_rowsel (every edge lane loads; out-of-range lanes read
# the row's last chunk) and lib_masked (its u16 kernels load out-of-range
# lanes from the frame start).  Then the regression test of §12.1.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_fuzzrep; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for v in product rowsel masked; do
    lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
    [ $v != product ] && lib=$PWD/tools/divergent/lib_$v.so
    AQZ_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "device_batch or stream" > $OUT/fuzz_${v}_$rep.log 2>&1
    rc=$?
    echo "$v rep $rep rc=$rc $(tail -1 $OUT/fuzz_${v}_$rep.log)"
    grep -h "AssertionError: case" $OUT/fuzz_${v}_$rep.log | cut -c1-200 | head -5
    [ $rc -le 1 ] || exit $rc
  done
done
# the divergent build over select loads, with forced-zero waitcnts
env AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2 \
  AQZ_LIB_PATH=$PWD/tools/divergent/lib_divselwz.so timeout -k 10 300 python -u tests/narrow_dbg.py --float-mean \
  > $OUT/dbg_divselwz.log 2>&1 || exit $?
echo "divselwz: $(tail -1 $OUT/dbg_divselwz.log)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_divergent.py -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/divergent_test.log 2>&1; echo "divergent test rc=$? $(tail -1 $OUT/divergent_test.log)"
echo "== done"
