#!/bin/bash
# Round 4, VERDICT r3 item 5 (512^2 u8 Decimate at 0.85 of its ceiling):
# units per wave.  Parity of the looped cascade kernel ($AQZ_UNITS_PER_WAVE=3:
# a remainder in every launch), then alternating A/B of 1/2/4 units per wave
# on the small-unit launches (512^2 u8, all methods) and the headline as a
# guard; plus the F-config load cache policy ($AQZ_LOAD_NT=0) A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_upw; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_UNITS_PER_WAVE=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py \
  tests/test_gpu_reference_vectors.py -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "batch or full_size or headline or digest or reference" > $OUT/upw_parity.log 2>&1 || { tail -30 $OUT/upw_parity.log; exit 1; }
tail -1 $OUT/upw_parity.log
b() { # tag env... -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc $BARGS \
    > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$tag', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for m in decimate mean max; do
    for u in 1 2 4; do
      BARGS="--workload 512x512_u8 --method $m" b "u8_512_${m}_upw$u" AQZ_UNITS_PER_WAVE=$u
    done
  done
  for u in 1 2; do
    BARGS="--workload 2048x2048_u16 --method decimate" b "u16_2048_decimate_upw$u" AQZ_UNITS_PER_WAVE=$u
    BARGS="--workload 4096x4096_u16 --method mean" b "headline_upw$u" AQZ_UNITS_PER_WAVE=$u
  done
  for nt in 1 0; do
    for m in max mean; do
      BARGS="--workload 4096x4096_f32 --method $m" b "f32_${m}_nt$nt" AQZ_LOAD_NT=$nt
    done
  done
done
echo "== done"
