#!/bin/bash
# Round 5: volume Decimate unit order (plane groups fastest, $AQZ_VOLUME_ZFAST)
# with the data in HBM (rotating buffer sets), 1 and 4 volumes per launch,
# three passes; the zfast launch checked against the oracle by the line.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_vzfast; mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2 3; do
  for b in 256 1024; do
    for z in 0 1; do
      timeout -k 10 200 env AQZ_VOLUME_ZFAST=$z python bench.py --workload 1024x1024x256_u16 --method decimate --batch $b \
        --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', 'planes $b', 'zfast $z', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
    done
  done
done
echo "== done"
