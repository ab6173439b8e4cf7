#!/bin/bash
# Round 5: config C1b (512^2 u8, 3 levels, 1024 frames) launcher knobs with
# the data in HBM (rotating buffer sets), two passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_c1bknobs; mkdir -p $OUT
export TMPDIR=/tmp
one() { # label, method, env...
  local lab=$1 m=$2; shift 2
  timeout -k 10 200 env "$@" python bench.py --workload 512x512_u8 --method $m --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', '$m', '$lab', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for pass in 1 2; do
  for m in mean max decimate; do
    one default $m AQZ_X=0
    one waves1 $m AQZ_CASCADE_WAVES=1
    one waves2 $m AQZ_CASCADE_WAVES=2
    one waves8 $m AQZ_CASCADE_WAVES=8
    one order1 $m AQZ_UNIT_ORDER=1
    one order2 $m AQZ_UNIT_ORDER=2
    one xcd $m AQZ_XCD_REMAP=1
  done
done
echo "== done"
