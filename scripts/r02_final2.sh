#!/bin/bash
# Round-2 closing validation: full GPU suite, C++ reference tests, smoke,
# the default bench line (PMC traffic, CPU baseline, e2e incl. blosc frames),
# rocprofv3 kernel stats of the headline, tiled headline.  gpurun_out/r02g/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02${RUN:-g}; mkdir -p $OUT
export TMPDIR=/tmp
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "== cpp"
for t in test_downsampler test_downsampler_odd_z; do
  timeout -k 10 120 tests/cpp/bin/$t > $OUT/$t.log 2>&1 || { tail -5 $OUT/$t.log; exit 1; }
  tail -1 $OUT/$t.log
done
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo "== headline bench (default)"
timeout -k 10 500 python bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_headline.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],r['traffic'],d['config']['check']);print(json.dumps(d['e2e']['blosc_frames']))"
echo "== rocprof headline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_headline -o run -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc \
  > $OUT/prof_headline.log 2>&1 || { tail -5 $OUT/prof_headline.log; exit 1; }
grep -o '"avg_launch_us": [0-9.]*' $OUT/prof_headline.log | head -1
echo "== tiled headline"
timeout -k 10 300 python bench.py --tiled --cpu-seconds 0 --e2e-frames 0 > $OUT/bench_tiled.json 2> $OUT/bench_tiled.err || { tail -20 $OUT/bench_tiled.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_tiled.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],r['traffic'])"
echo "== segmented band shape"
timeout -k 10 300 python bench.py --shape 8704x2040 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/bench_8704.json 2> $OUT/bench_8704.err || { tail -20 $OUT/bench_8704.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_8704.json'));r=d['roofline'];print('8704x2040',d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],d['config']['check'])"
echo "== done"
