#!/bin/bash
# Round 3: misaligned segments, second look at the shapes where they won in
# r03_misseg.sh (wide f32, u8) and at neighbours, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_misseg2; mkdir -p $OUT
export TMPDIR=/tmp
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 5472x3648 6000x4000 4100x4100 4500x3000; do
    for s in 0 4; do
      b f32_$sh "AQZ_BAND_MIS_SEG=$s" --workload 4096x4096_f32 --shape $sh
    done
  done
  for sh in 5472x3648 6000x4000 7000x5000; do
    for s in 0 2 4; do
      b u8_$sh "AQZ_BAND_MIS_SEG=$s" --workload 512x512_u8 --chunk 256 --shape $sh
    done
  done
  for sh in 6000x4000 5472x3648; do
    for s in 0 4; do
      b u16_$sh "AQZ_BAND_MIS_SEG=$s" --shape $sh
    done
  done
done
echo "== done"
