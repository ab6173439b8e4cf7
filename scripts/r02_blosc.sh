#!/bin/bash
# Round-2 GPU session: blosc frames of device chunks vs c-blosc, full GPU
# suite, smoke, headline bench + rocprof stats, chunk-compression bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02b; mkdir -p $OUT
export TMPDIR=/tmp
echo "== blosc gpu tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_blosc.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_blosc.log 2>&1 || { tail -40 $OUT/pytest_blosc.log; exit 1; }
tail -3 $OUT/pytest_blosc.log
echo "== blosc bench"
timeout -k 10 300 python -u tools/blosc_bench.py > $OUT/blosc_bench.jsonl 2> $OUT/blosc_bench.err || { tail -20 $OUT/blosc_bench.err; exit 1; }
cat $OUT/blosc_bench.jsonl
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
echo "== headline bench"
timeout -k 10 400 python bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
head -c 700 $OUT/bench_headline.json; echo
echo "== rocprof headline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_headline -o run -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc \
  > $OUT/prof_headline.log 2>&1 || { tail -5 $OUT/prof_headline.log; exit 1; }
grep -o '"avg_launch_us": [0-9.]*' $OUT/prof_headline.log | head -1
echo "== done"
