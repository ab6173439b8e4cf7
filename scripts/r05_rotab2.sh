#!/bin/bash
# Round 5: with rotating buffer sets, (1) a second pass of the 512^2 u8
# Mean/Max units-per-wave and load-policy choices, (2) the chunk-tiled
# launches' plain-load rule for small units against nontemporal loads.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_rotab2; mkdir -p $OUT
export TMPDIR=/tmp
one() { # label, workload, method, extra bench args (quoted), env...
  local lab=$1 w=$2 m=$3 xa=$4; shift 4
  timeout -k 10 200 env "$@" python bench.py --workload $w --method $m --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 --no-pmc $xa > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', '$w', '$m', '$lab', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for pass in 2 3; do
  for m in mean max; do for u in 0 1; do for nt in -1 0; do
    one "upw$u nt$nt" 512x512_u8 $m "" AQZ_UNITS_PER_WAVE=$u AQZ_LOAD_NT=$nt
  done; done; done
  for w in 512x512_u8 2048x2048_u16; do for m in decimate mean; do for nt in -1 1; do
    one "tiled nt$nt" $w $m "--tiled" AQZ_LOAD_NT=$nt
  done; done; done
done
echo "== done"
