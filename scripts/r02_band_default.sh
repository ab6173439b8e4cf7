#!/bin/bash
# Round-2: 8-wave staged bands on by default for aligned 5-8-tile bands.
# Full GPU suite, then default vs $AQZ_BAND_ALIGNED=0 on the affected shapes,
# then the default bench line (PMC traffic) and rocprof stats.  gpurun_out/r02k/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02k; mkdir -p $OUT
export TMPDIR=/tmp
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
LOG=$OUT/band_default_ab.log; : > $LOG
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
for rep in 1 2; do
  for w in "" "--shape 3072x3072" "--workload 4096x4096_f32"; do
    read -ra A <<< "$w"
    run direct AQZ_BAND_ALIGNED=0 -- "${A[@]}"
    run staged X=0 -- "${A[@]}"
  done
done
echo "== default bench line"
timeout -k 10 500 python bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_headline.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],r['traffic'],d['config']['check'])"
echo "== rocprof headline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_headline -o run -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc \
  > $OUT/prof_headline.log 2>&1 || { tail -5 $OUT/prof_headline.log; exit 1; }
grep -o '"avg_launch_us": [0-9.]*' $OUT/prof_headline.log | head -1
head -3 $OUT/prof_headline/run_kernel_stats.csv | cut -c1-160
echo "== done"
