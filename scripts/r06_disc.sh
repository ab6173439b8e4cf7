#!/bin/bash
# Round 6: waits or spacing?  Both edge-tile faults rerun
# on builds whose instruction order is unchanged: load waits forced to zero
# (-amdgpu-waitcnt-load-forcezero) or an s_nop before every instruction
# (-amdgpu-snop-padding=1).  u16 select form: fuzz case 181, 400 launches in
# one process; f32 divergent form: the 18 float Mean cases under round 5's
# launch, three times.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_disc; mkdir -p $OUT
for v in u16rowsel u16rowselldz u16rowselpad; do
  AQZ_LIB_PATH=$PWD/tools/divergent/lib_$v.so timeout -k 10 200 python -u tests/fuzz_repeat.py --cases 181 --reps 400 \
    > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  echo "$v: $(cat $OUT/$v.json)" | tee -a $OUT/summary.txt
done
for v in div divldz divpad; do
  for rep in 1 2 3; do
    env AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2 \
      AQZ_LIB_PATH=$PWD/tools/divergent/lib_$v.so timeout -k 10 200 python -u tests/narrow_dbg.py --float-mean \
      > $OUT/${v}_$rep.log 2>&1 || { tail -5 $OUT/${v}_$rep.log; exit 1; }
    echo "$v rep $rep: $(tail -1 $OUT/${v}_$rep.log)" | tee -a $OUT/summary.txt
  done
done
echo "== done"
