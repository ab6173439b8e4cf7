#!/bin/bash
# Round 5: load policy and units per wave of the small-unit launches (C1b,
# C2, V), re-checked with rotating buffer sets (data in HBM, not in the
# Infinity Cache).  Two passes; prints us per launch and fraction of spec.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_rotab; mkdir -p $OUT
export TMPDIR=/tmp
one() { # label, workload, method, env...
  local lab=$1 w=$2 m=$3; shift 3
  timeout -k 10 200 env "$@" python bench.py --workload $w --method $m --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', '$w', '$m', '$lab', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for pass in ${PASSES:-1 2}; do
  for u in 0 1 2 4 8; do for nt in -1 0 1; do
    one "upw$u nt$nt" 512x512_u8 decimate AQZ_UNITS_PER_WAVE=$u AQZ_LOAD_NT=$nt
  done; done
  for m in mean max; do for u in 0 1 2 4; do for nt in -1 0; do
    one "upw$u nt$nt" 512x512_u8 $m AQZ_UNITS_PER_WAVE=$u AQZ_LOAD_NT=$nt
  done; done; done
  for m in decimate mean; do for u in 0 2; do for nt in -1 0 1; do
    one "upw$u nt$nt" 2048x2048_u16 $m AQZ_UNITS_PER_WAVE=$u AQZ_LOAD_NT=$nt
  done; done; done
  for u in 1 2; do for nt in 0 1; do
    one "vupw$u vnt$nt" 1024x1024x256_u16 decimate AQZ_VOLUME_UPW=$u AQZ_VOLUME_NT=$nt
  done; done
done
echo "== done"
