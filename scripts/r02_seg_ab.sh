#!/bin/bash
# Round-2 A/B: aligned bands wider than 8 tiles staged in 8-tile segments
# ($AQZ_BAND_SEGMENTS=1) against direct stores and the tiled kernel; box check
# on the headline (direct vs staged 8-wave bands).  gpurun_out/r02n/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02n; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
LOG=$OUT/seg_ab.log; : > $LOG
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 --no-pmc "$@" > $OUT/one.json 2> $OUT/one.err || { tail -5 $OUT/one.err; exit 1; }
  OUTJ=$OUT/one.json python - "$name" "$*" >> $LOG <<'PY'
import json, os, sys
d = json.load(open(os.environ["OUTJ"])); r = d["roofline"]
print(f"{sys.argv[2]:<36} {sys.argv[1]:<8} {r['avg_launch_us']:9.1f} us  frac {r['frac']:.4f}  ceil {r['same_mix_ceiling']['frac_of_ceiling']:.4f}  {d['config']['check']}")
PY
  tail -1 $LOG
}
for rep in 1 2; do
  run direct AQZ_BAND_ALIGNED=0 --
  run staged X=0 --
  for w in "--shape 8192x2048" "--shape 8704x2040" "--shape 6144x3072" "--workload 4096x4096_f32 --shape 8192x2048"; do
    read -ra A <<< "$w"
    run direct X=0 -- "${A[@]}"
    run segs AQZ_BAND_SEGMENTS=1 -- "${A[@]}"
    run tiled X=0 -- "${A[@]}" --tiled
  done
done
echo "== done"
