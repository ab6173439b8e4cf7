#!/bin/bash
# Round 5: C1b (512^2 u8) Min/Max units per wave and load hint (env only).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_u8minmax; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local label=$1 m=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload 512x512_u8 --method $m --steps 30 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for m in min max mean; do
    run ${m}_default_r$rep $m AQZ_UNUSED=0
    run ${m}_upw1_r$rep $m AQZ_UNITS_PER_WAVE=1
    run ${m}_upw4_r$rep $m AQZ_UNITS_PER_WAVE=4
    run ${m}_plain_r$rep $m AQZ_LOAD_NT=0
    run ${m}_upw4_plain_r$rep $m AQZ_UNITS_PER_WAVE=4 AQZ_LOAD_NT=0
  done
done
echo "== done"
