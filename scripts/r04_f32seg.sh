#!/bin/bash
# Round 4: F config segment sizes (2 vs 4 tiles) for every method, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_f32seg; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for m in max min mean; do
    for n in 4 2; do
      AQZ_BAND_SEGN=$n timeout -k 10 300 python bench.py --workload 4096x4096_f32 --method $m --steps 20 --warmup 5 \
        --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('segn=$n', '$m', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
    done
  done
done
echo "== done"
