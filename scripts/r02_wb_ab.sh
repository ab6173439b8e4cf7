#!/bin/bash
# Round-2 A/B: write-back row-major level stores ($AQZ_STORE_WB level mask)
# with and without the XCD-contiguous block order ($AQZ_XCD_REMAP), on the
# headline and on frames whose level rows split 64-B bursts.  Alternating
# runs on one box; one JSON summary line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02f; mkdir -p $OUT
LOG=$OUT/wb_ab.log; : > $LOG
run() {  # name env... -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc --no-check "$@" > $OUT/one.json 2> $OUT/one.err || { tail -5 $OUT/one.err; exit 1; }
  python - "$name" "$*" >> $LOG <<'PY'
import json, sys
d = json.load(open("gpurun_out/r02f/one.json")); r = d["roofline"]
print(f"{sys.argv[2]:<28} {sys.argv[1]:<16} {r['avg_launch_us']:9.1f} us  frac {r['frac']:.4f}  ceil {r['same_mix_ceiling']['frac_of_ceiling']:.4f}  {d['config']['batch_path']}")
PY
  tail -1 $LOG
}
for rep in 1 2; do
  for shape in "" "--shape 3000x3000" "--shape 5472x3648" "--shape 4100x4100" "--shape 2600x2600"; do
    run base AQZ_STORE_WB=0 AQZ_XCD_REMAP=0 -- $shape
    run remap AQZ_STORE_WB=0 AQZ_XCD_REMAP=1 -- $shape
    run wb AQZ_STORE_WB=15 AQZ_XCD_REMAP=0 -- $shape
    run wb+remap AQZ_STORE_WB=15 AQZ_XCD_REMAP=1 -- $shape
  done
  for shape in "--shape 2000x2000" "--shape 1500x1500"; do
    run band AQZ_STORE_WB=0 AQZ_XCD_REMAP=0 -- $shape
    run nb-base AQZ_BAND_STAGING=0 AQZ_STORE_WB=0 AQZ_XCD_REMAP=0 -- $shape
    run nb-wb+remap AQZ_BAND_STAGING=0 AQZ_STORE_WB=15 AQZ_XCD_REMAP=1 -- $shape
  done
done
echo "== done"
