#!/bin/bash
# Round 4: row-major camera frames — segment width and storing waves of the
# misaligned band kernel ($AQZ_BAND_MIS_SEG, $AQZ_BAND_LAST), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_misseg; mkdir -p $OUT
export TMPDIR=/tmp
b() { # tag shape env...
  local tag=$1 sh=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --shape $sh --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc \
    > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$tag', '$sh', r['avg_launch_us'], r['frac'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 6000x4000 5472x3648; do
    b default $sh
    b seg3 $sh AQZ_BAND_MIS_SEG=3
    b seg6 $sh AQZ_BAND_MIS_SEG=6
    b seg8 $sh AQZ_BAND_MIS_SEG=8
    b seg4_last2 $sh AQZ_BAND_LAST=2
  done
  for sh in 3000x3000 2600x2600 2000x2000; do
    b default $sh
    b last2 $sh AQZ_BAND_LAST=2
    b seg3 $sh AQZ_BAND_MIS_SEG=3
  done
done
echo "== done"
