#!/bin/bash
# Round-2 profile set: headline (row-major, the BASELINE metric) and
# chunk-tiled benches with PMC traffic, rocprofv3 kernel stats of both, and
# every BASELINE config.  Outputs under gpurun_out/r02/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02; mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $1"; }
step "headline"
timeout -k 10 400 python bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
head -c 600 $OUT/bench_headline.json; echo
step "tiled headline"
timeout -k 10 400 python bench.py --tiled --cpu-seconds 0 --e2e-frames 0 > $OUT/bench_tiled_headline.json 2> $OUT/bench_tiled_headline.err || { tail -20 $OUT/bench_tiled_headline.err; exit 1; }
head -c 600 $OUT/bench_tiled_headline.json; echo
for mode in "" "--tiled"; do
  name=prof_headline${mode:+_tiled}
  step "rocprof $name"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc $mode \
    > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  grep -o '"avg_launch_us": [0-9.]*' $OUT/$name.log | head -1
done
step "configs"
for w in 4096x4096_f32 2048x2048_u16 512x512_u8 1024x1024x256_u16; do
  timeout -k 10 300 python bench.py --workload $w --cpu-seconds 5 > $OUT/sweep_$w.json 2> $OUT/sweep_$w.err || { tail -20 $OUT/sweep_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sweep_$w.json'));r=d['roofline'];print('$w',d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'),r['traffic'])"
done
echo "== done"
