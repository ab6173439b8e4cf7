#!/bin/bash
# A/B: volume Decimate with 16 vs 32 bytes per lane ($AQZ_VOLUME_WIDE), config V.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 40 --warmup 5 --workload 1024x1024x256_u16 --method decimate"
for rep in 1 2 3; do for w in 0 1; do
  AQZ_VOLUME_WIDE=$w timeout -k 10 200 python bench.py $B > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('wide=$w',d['value'],d['config']['check'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))" | tee -a $OUT/volwide_ab.log
done; done
echo "== done"
