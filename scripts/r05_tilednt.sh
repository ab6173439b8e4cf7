#!/bin/bash
# Round 5: the chunk-tiled cascade's load hint under Decimate and Mean
# (AQZ_LOAD_NT=0 against the default), the 2-D BASELINE sizes, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_tilednt; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local label=$1 w=$2 m=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --workload $w --method $m --tiled --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for w in 4096x4096_u16 4096x4096_f32 2048x2048_u16 512x512_u8; do
    for m in decimate mean; do
      run t_${w}_${m}_default_r$rep $w $m AQZ_UNUSED=0
      run t_${w}_${m}_plain_r$rep $w $m AQZ_LOAD_NT=0
    done
  done
done
echo "== done"
