#!/bin/bash
# Round 3: u16 Min/Max band kernels held to 80 VGPRs (6 waves per SIMD
# instead of 5, amdgpu_waves_per_eu) against the tree without the hint
# (_ab_old/), same box, alternating, two rounds; GPU parity of the band
# kernels first.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out/r03_wpe2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -q -x -k "device_batch or headline or fuzz" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
b() { # label dir args...
  local lab=$1 d=$2; shift 2
  (cd $d && timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err) || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$(basename $d)', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for d in $ROOTDIR $ROOTDIR/_ab_old; do
    b headline_min $d --method min
    b headline_max $d --method max
    b c2_min $d --workload 2048x2048_u16 --method min
    b u16_3000_max $d --shape 3000x3000 --method max
    b u16_2304_max $d --shape 2304x2304 --method max
    b headline $d
  done
done
echo "== done"
