#!/bin/bash
# Round 5: aligned 4-tile row bands staged in LDS (the new default) against
# direct stores ($AQZ_BAND_ALIGNED=0, the old 4-tile path) on the BASELINE
# C2 config and other 4-tile shapes, data in HBM (rotating buffer sets).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_band4; mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2; do
  for ws in "2048x2048_u16 -" "512x512_u8 4096x4096" "4096x4096_f32 2048x2048" "4096x4096_u32 2048x2048"; do
    set -- $ws
    xa=""; [ "$2" = "-" ] || xa="--shape $2"
    for m in mean max decimate; do
      for al in 1 0; do
        timeout -k 10 200 env AQZ_BAND_ALIGNED=$al python bench.py --workload $1 $xa --method $m --steps 20 --warmup 5 \
          --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', '$1', '$2', '$m', 'aligned_staging=$al', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
      done
    done
  done
done
echo "== done"
