#!/bin/bash
# Round 6, second probe round on the round-5 divergent-branch failure (under
# round 5's launch, scripts/r06_divergent2.sh): the product's wave-uniform
# form with forced-zero waitcnts (does the product's edge path fail under
# the same timing?), the divergent form with select loads on edge tiles
# (no exec-masked loads), and with a printf on in-range edge chunks that
# load as all-zero bits; the product three times (robustness).  Then the
# four-units-per-wave V Decimate A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_divergent3; mkdir -p $OUT
export TMPDIR=/tmp
R5="AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2"
for v in prodwz divsel divdbg product product product; do
  lib=$PWD/tools/divergent/lib_$v.so
  [ $v = product ] && lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
  [ -f $lib ] || { echo "== $v: not built"; continue; }
  env $R5 AQZ_LIB_PATH=$lib timeout -k 10 300 python -u tests/narrow_dbg.py >> $OUT/dbg_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep "differing" $OUT/dbg_$v.log | tail -12
  [ $rc -eq 0 ] || exit $rc
done
[ -f $OUT/dbg_divdbg.log ] && { grep -c AQZDBG $OUT/dbg_divdbg.log; grep AQZDBG $OUT/dbg_divdbg.log | head -20; }
for rep in 1 2; do
  for u in 2 4; do
    for b in 1024 256; do
      AQZ_VOLUME_UPW=$u timeout -k 10 300 python bench.py --workload 1024x1024x256_u16 --method decimate --batch $b \
        --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/v_upw${u}_b${b}_$rep.json 2> $OUT/v_upw${u}_b${b}_$rep.err \
        || { tail -20 $OUT/v_upw${u}_b${b}_$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/v_upw${u}_b${b}_$rep.json'));r=d['roofline'];print('upw $u planes $b rep $rep', r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])"
    done
  done
done
echo "== done"
