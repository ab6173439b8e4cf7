#!/bin/bash
# Round-2 A/B of the row-major cascade's unit mapping on whatever box this is
# ("slow" boxes run the row-major headline ~15% slower than the tiled one):
# unit order ($AQZ_UNIT_ORDER), waves per workgroup ($AQZ_CASCADE_WAVES), the
# XCD-contiguous order ($AQZ_XCD_REMAP); the tiled headline for reference.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02h; mkdir -p $OUT
LOG=$OUT/order_ab.log; : > $LOG
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc --no-check "$@" > $OUT/one.json 2> $OUT/one.err || { tail -5 $OUT/one.err; exit 1; }
  python - "$name" "$*" >> $LOG <<'PY'
import json, sys
d = json.load(open("gpurun_out/r02h/one.json")); r = d["roofline"]
print(f"{sys.argv[2]:<30} {sys.argv[1]:<14} {r['avg_launch_us']:9.1f} us  frac {r['frac']:.4f}  ceil {r['same_mix_ceiling']['frac_of_ceiling']:.4f}")
PY
  tail -1 $LOG
}
for rep in 1 2; do
  for w in "" "--workload 4096x4096_f32" "--shape 3000x3000"; do
    run base X=0 -- $w
    run remap AQZ_XCD_REMAP=1 -- $w
    run order1 AQZ_UNIT_ORDER=1 -- $w
    run order2 AQZ_UNIT_ORDER=2 -- $w
    run waves8 AQZ_CASCADE_WAVES=8 -- $w
    run waves8+remap AQZ_CASCADE_WAVES=8 AQZ_XCD_REMAP=1 -- $w
    run waves2 AQZ_CASCADE_WAVES=2 -- $w
    run tiled X=0 -- $w --tiled
  done
done
echo "== done"
