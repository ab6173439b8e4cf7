#!/bin/bash
# Round 6: the f32 divergent form with LLVM's VGPR
# live-range optimisation for if-else regions off
# (-amdgpu-opt-vgpr-liverange=false), and with early if-conversion off,
# against the unchanged divergent build: the 18 float Mean cases under
# round 5's launch, three times each.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_nolr; mkdir -p $OUT
for v in div divnolr divnoifcvt; do
  [ -f tools/divergent/lib_$v.so ] || { echo "$v: not built"; continue; }
  for rep in 1 2 3; do
    env AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2 \
      AQZ_LIB_PATH=$PWD/tools/divergent/lib_$v.so timeout -k 10 200 python -u tests/narrow_dbg.py --float-mean \
      > $OUT/${v}_$rep.log 2>&1 || { tail -5 $OUT/${v}_$rep.log; exit 1; }
    echo "$v rep $rep: $(tail -1 $OUT/${v}_$rep.log)" | tee -a $OUT/summary.txt
  done
done
echo "== done"
