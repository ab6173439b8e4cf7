#!/bin/bash
# Round 6: launch-knob scan on the two launches furthest below their
# ceilings, C1b Decimate (512^2 u8, 3 levels) and V Decimate at one volume
# per launch; every line rotated into HBM, bit-exact check on.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_knobs; mkdir -p $OUT
run() { # tag env... -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc \
    > $OUT/$tag.json 2> $OUT/$tag.err || { tail -5 $OUT/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));r=d['roofline'];print('$tag', r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'][:9])" | tee -a $OUT/knobs.log
}
for rep in 1 2; do
  C1B="--workload 512x512_u8 --method decimate"
  run c1b_default_$rep X=0 -- $C1B || exit 1
  run c1b_waves8_$rep AQZ_CASCADE_WAVES=8 -- $C1B || exit 1
  run c1b_waves2_$rep AQZ_CASCADE_WAVES=2 -- $C1B || exit 1
  run c1b_upw8_$rep AQZ_UNITS_PER_WAVE=8 -- $C1B || exit 1
  run c1b_order2_$rep AQZ_UNIT_ORDER=2 -- $C1B || exit 1
  run c1b_remap_$rep AQZ_XCD_REMAP=1 -- $C1B || exit 1
  V1="--workload 1024x1024x256_u16 --batch 256 --method decimate"
  run v1_default_$rep X=0 -- $V1 || exit 1
  run v1_nt0_$rep AQZ_VOLUME_NT=0 -- $V1 || exit 1
  run v1_upw1_$rep AQZ_VOLUME_UPW=1 -- $V1 || exit 1
  run v1_zfast0_$rep AQZ_VOLUME_ZFAST=0 -- $V1 || exit 1
done
echo "== done"
