#!/bin/bash
# Round 5: headline launch size — frames per step 32 / 64 / 128 / 256,
# twice (the tail of each launch is amortised over more frames).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_batch; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for b in 32 64 128 256; do
    timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc \
      > $OUT/b${b}_r$rep.json 2> $OUT/b${b}_r$rep.err || { tail -20 $OUT/b${b}_r$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b${b}_r$rep.json'));r=d['roofline'];print('b$b r$rep', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))" | tee -a $OUT/ab.log
  done
done
echo "== done"
