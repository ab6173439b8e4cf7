#!/bin/bash
# Round-2 A/B: row bands of up to 8 waves staged in LDS for aligned frames
# ($AQZ_BAND_FORCE level mask) against direct stores and the tiled kernel, on
# whatever box this is.  SHAPES: ';'-separated bench argument sets ("" = the
# headline); RUN: output suffix.  Alternating runs, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02${RUN:-i}; mkdir -p $OUT
LOG=$OUT/band_ab.log; : > $LOG
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc "$@" > $OUT/one.json 2> $OUT/one.err || { tail -5 $OUT/one.err; exit 1; }
  OUTJ=$OUT/one.json python - "$name" "$*" >> $LOG <<'PY'
import json, os, sys
d = json.load(open(os.environ["OUTJ"])); r = d["roofline"]
print(f"{sys.argv[2]:<30} {sys.argv[1]:<8} {r['avg_launch_us']:9.1f} us  frac {r['frac']:.4f}  ceil {r['same_mix_ceiling']['frac_of_ceiling']:.4f}  {d['config']['check']}")
PY
  tail -1 $LOG
}
IFS=';' read -ra SETS <<< "${SHAPES:-;--workload 2048x2048_u16;--workload 4096x4096_f32}"
for rep in 1 2; do
  for w in "${SETS[@]}"; do
    read -ra A <<< "$w"
    run base X=0 -- "${A[@]}"
    run band15 AQZ_BAND_FORCE=15 -- "${A[@]}"
    run tiled X=0 -- "${A[@]}" --tiled
  done
done
echo "== done"
