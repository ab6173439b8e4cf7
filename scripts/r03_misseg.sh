#!/bin/bash
# Round 3: misaligned bands wider than one wave may store, in balanced
# segments of <= $AQZ_BAND_MIS_SEG tiles, each staged and stored by its last
# wave.  Parity for 2, 3 and 4, then A/B against direct stores (0).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_misseg; mkdir -p $OUT
export TMPDIR=/tmp
for s in 2 3 4; do
  AQZ_BAND_MIS_SEG=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch or headline" --timeout 120 --timeout-method thread > $OUT/pytest_seg$s.log 2>&1 || { tail -30 $OUT/pytest_seg$s.log; exit 1; }
  tail -1 $OUT/pytest_seg$s.log
done
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1; do
  for sh in 4000x3000 5472x3648 4100x4100 6000x4000; do
    for s in 0 2 3 4; do
      b u16_$sh "AQZ_BAND_MIS_SEG=$s" --shape $sh
    done
  done
  for s in 0 2 3 4; do
    b f32_3000x3000 "AQZ_BAND_MIS_SEG=$s" --workload 4096x4096_f32 --shape 3000x3000
    b f32_5472x3648 "AQZ_BAND_MIS_SEG=$s" --workload 4096x4096_f32 --shape 5472x3648
    b u8_5000x4000 "AQZ_BAND_MIS_SEG=$s" --workload 512x512_u8 --chunk 256 --shape 5000x4000
    b u8_5472x3648 "AQZ_BAND_MIS_SEG=$s" --workload 512x512_u8 --chunk 256 --shape 5472x3648
  done
done
echo "== done"
