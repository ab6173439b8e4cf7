#!/bin/bash
# Round 5: config C2 (2048^2 u16, 4 levels, 64 frames) launcher knobs with
# the data in HBM (rotating buffer sets), two passes; plus the rotation
# target itself (1 GiB default against 4 GiB) on the small-read-set configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_c2knobs; mkdir -p $OUT
export TMPDIR=/tmp
one() { # label, workload, method, extra args, env...
  local lab=$1 w=$2 m=$3 xa=$4; shift 4
  timeout -k 10 200 env "$@" python bench.py --workload $w --method $m --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 --no-pmc $xa > $OUT/cur.json 2> $OUT/cur.err || { tail -20 $OUT/cur.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/cur.json'));r=d['roofline'];print('$pass', '$w', '$m', '$lab', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for pass in 1 2; do
  for m in mean decimate; do
    one default 2048x2048_u16 $m "" AQZ_X=0
    one force7 2048x2048_u16 $m "" AQZ_BAND_FORCE=7
    one waves2 2048x2048_u16 $m "" AQZ_CASCADE_WAVES=2
    one waves8 2048x2048_u16 $m "" AQZ_CASCADE_WAVES=8
    one order1 2048x2048_u16 $m "" AQZ_UNIT_ORDER=1
    one order2 2048x2048_u16 $m "" AQZ_UNIT_ORDER=2
    one xcd 2048x2048_u16 $m "" AQZ_XCD_REMAP=1
    one wb7 2048x2048_u16 $m "" AQZ_STORE_WB=7
    one rot4g 2048x2048_u16 $m "--rotate-mib 4096" AQZ_X=0
  done
  one rot4g 512x512_u8 mean "--rotate-mib 4096" AQZ_X=0
  one rot4g 512x512_u8 decimate "--rotate-mib 4096" AQZ_X=0
  one rot4g 1024x1024x256_u16 decimate "--rotate-mib 4096" AQZ_X=0
  one rot4g 1024x1024x256_u16 mean "--rotate-mib 4096" AQZ_X=0
done
echo "== done"
