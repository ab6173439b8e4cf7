#!/bin/bash
# Round 6: the product's fuzz suite (every dtype, method and store scheme)
# under other launch rules than the defaults, twice each: round 5's launch,
# and single A/B knobs that move frames between kernels and store schemes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_knobparity; mkdir -p $OUT
i=0
while read -r cfg; do
  i=$((i+1))
  for rep in 1 2; do
    env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $OUT/cfg${i}_$rep.log 2>&1
    rc=$?
    echo "[$cfg] rep $rep rc=$rc $(tail -1 $OUT/cfg${i}_$rep.log)" | tee -a $OUT/summary.txt
    grep -h "AssertionError: case" $OUT/cfg${i}_$rep.log | cut -c1-200 | head -3 | tee -a $OUT/summary.txt
    [ $rc -le 1 ] || exit $rc
  done
done <<'CFGS'
AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2
AQZ_CASCADE_NARROW=1
AQZ_CASCADE_NARROW=0
AQZ_BAND_STAGING=0
AQZ_BAND_LAST=2
AQZ_UNITS_PER_WAVE=4
AQZ_CASCADE_WAVES=8
AQZ_XCD_REMAP=1
CFGS
echo "== done"
