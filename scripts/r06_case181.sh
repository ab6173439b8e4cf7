#!/bin/bash
# Round 6: fuzz case 181 (u16 Mean 4009x30, 3 levels, misaligned band kernel
# stored by its last wave) failed once on the row-local edge-load form: the
# frame's last level-1 pixel.  Is it the change or a race?  The same case
# three times on the product, twice on lib_masked (its u16 kernels are the
# previous, frame-start form), then the fuzz test alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_case181; mkdir -p $OUT
export TMPDIR=/tmp
for v in product product product masked masked; do
  lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
  [ $v = masked ] && lib=$PWD/tools/divergent/lib_masked.so
  AQZ_LIB_PATH=$lib timeout -k 10 300 python -u tests/narrow_dbg.py --cases 181,153,25,51 >> $OUT/dbg_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "differing|TOTAL" $OUT/dbg_$v.log | tail -4
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "181" > $OUT/fuzz181.log 2>&1; echo "fuzz 181 rc=$? $(tail -1 $OUT/fuzz181.log)"
echo "== done"
