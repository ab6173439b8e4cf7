#!/bin/bash
# Round 3: final misaligned-band policy (last-wave stores for bands of <= 4
# tiles, <= 6 for 2-byte types) against the policy before it (barrier-staged
# bands of <= 4 tiles, direct stores above).  Full GPU suite first.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_mis_confirm; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
OLD="AQZ_BAND_MIS_MAX=4 AQZ_BAND_LAST=0"
for i in 1 2; do
  for sh in 2000x2000 2304x2304 2600x2600 3000x3000 5472x3648; do
    b u16_$sh "X=0" --shape $sh
    b u16_$sh "$OLD" --shape $sh
  done
  b f32_3000x3000 "X=0" --workload 4096x4096_f32 --shape 3000x3000
  b f32_2000x2000 "X=0" --workload 4096x4096_f32 --shape 2000x2000
  b f32_2000x2000 "$OLD" --workload 4096x4096_f32 --shape 2000x2000
  b u8_3000x3000 "X=0" --workload 512x512_u8 --chunk 256 --shape 3000x3000
  b u8_3000x3000 "$OLD" --workload 512x512_u8 --chunk 256 --shape 3000x3000
  b u8_5000x4000 "X=0" --workload 512x512_u8 --chunk 256 --shape 5000x4000
  b headline "X=0"
  b f32 "X=0" --workload 4096x4096_f32
done
echo "== done"
