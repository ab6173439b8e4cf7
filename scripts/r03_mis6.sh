#!/bin/bash
# Round 3: misaligned bands.  New default: bands of <= 6 tiles staged and
# stored by their last wave.  Edge mode ($AQZ_BAND_EDGES=1): each wave stores
# the bursts inside its own tile from registers, the last wave only the
# shared ones.  Against the policy before (barrier-staged bands of <= 4
# tiles, direct stores above: AQZ_BAND_MIS_MAX=4 AQZ_BAND_LAST=0).  Full GPU
# suite first, then parity of the edge variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_mis6; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
AQZ_BAND_EDGES=1 AQZ_BAND_MIS_MAX=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch or headline" --timeout 120 --timeout-method thread > $OUT/pytest_edges.log 2>&1 || { tail -30 $OUT/pytest_edges.log; exit 1; }
tail -1 $OUT/pytest_edges.log
AQZ_BAND_EDGES=1 AQZ_BAND_FORCE=15 AQZ_BAND_LAST=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch" --timeout 120 --timeout-method thread > $OUT/pytest_edges_barrier.log 2>&1 || { tail -30 $OUT/pytest_edges_barrier.log; exit 1; }
tail -1 $OUT/pytest_edges_barrier.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
OLD="AQZ_BAND_MIS_MAX=4 AQZ_BAND_LAST=0"
EDG="AQZ_BAND_EDGES=1 AQZ_BAND_MIS_MAX=8"
for i in 1; do
  for sh in 1000x1000 2000x2000 2600x2600 3000x3000 4000x3000 2304x2304; do
    b u16_$sh "X=0" --shape $sh
    b u16_$sh "$EDG" --shape $sh
    b u16_$sh "$OLD" --shape $sh
  done
  for sh in 2000x2000 3000x3000; do
    b f32_$sh "X=0" --workload 4096x4096_f32 --shape $sh
    b f32_$sh "$EDG" --workload 4096x4096_f32 --shape $sh
    b f32_$sh "$OLD" --workload 4096x4096_f32 --shape $sh
  done
  for sh in 3000x3000 5000x4000; do
    b u8_$sh "X=0" --workload 512x512_u8 --chunk 256 --shape $sh
    b u8_$sh "$EDG" --workload 512x512_u8 --chunk 256 --shape $sh
    b u8_$sh "$OLD" --workload 512x512_u8 --chunk 256 --shape $sh
  done
  b headline "X=0"
done
echo "== done"
