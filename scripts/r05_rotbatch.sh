#!/bin/bash
# Round 5: launch size of the small-frame configs with the data in HBM
# (rotating buffer sets): C2 64/128/256 frames, C1b 1024/4096/8192 frames,
# V 1 and 2 volumes per launch; Mean and Decimate, two passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_rotbatch; mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2; do
  for wb in "2048x2048_u16 64" "2048x2048_u16 128" "2048x2048_u16 256" "512x512_u8 1024" "512x512_u8 4096" "512x512_u8 8192" "1024x1024x256_u16 256" "1024x1024x256_u16 512"; do
    set -- $wb
    for m in mean decimate; do
      timeout -k 10 200 python bench.py --workload $1 --batch $2 --method $m --steps 20 --warmup 5 \
        --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', '$1', '$2', '$m', r['buffer_sets'], r['avg_launch_us'], round(r['avg_launch_us']/$2, 4), r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
    done
  done
done
echo "== done"
