#!/bin/bash
# Round 6: reproduce the round-5 divergent-branch failure.  Round 5's launch
# rules put these fuzz cases on 16-byte f32 tiles in band workgroups of the
# direct-store cascade_kernel with two units per wave (Mean took 2 units of
# < 4 KiB then); today's defaults take other kernels.  The env below restores
# that launch; each library variant (tools/divergent/build.sh) runs
# tests/narrow_dbg.py's four cases under it.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_divergent2; mkdir -p $OUT
export TMPDIR=/tmp
R5="AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2"
for v in product div wz nopre nosink; do
  lib=$PWD/tools/divergent/lib_$v.so
  [ $v = product ] && lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
  env $R5 AQZ_LIB_PATH=$lib timeout -k 10 300 python -u tests/narrow_dbg.py > $OUT/dbg_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep "differing" $OUT/dbg_$v.log
  [ $rc -eq 0 ] || exit $rc
done
# the same with one unit per wave (only AQZ_UNITS_PER_WAVE differs)
env AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=1 \
  AQZ_LIB_PATH=$PWD/tools/divergent/lib_div.so timeout -k 10 300 python -u tests/narrow_dbg.py > $OUT/dbg_div_upw1.log 2>&1
echo "== div upw1 rc=$?"; grep "differing" $OUT/dbg_div_upw1.log
# the default bench line on this library (e2e: C++ caller overlap, node drop-in)
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));e=d['e2e'];print(d['value'], d['roofline']['frac'], json.dumps(e.get('async_overlap')), json.dumps(e.get('node'))[:600])"
echo "== done"
