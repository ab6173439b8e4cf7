#!/bin/bash
# Round-2 GPU session: chunk-lattice batches (parity vs oracle, blosc of whole
# chunks), tiled regression tests, tiled/row-major headline after the change.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02c; mkdir -p $OUT
export TMPDIR=/tmp
echo "== lattice tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lattice.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_lattice.log 2>&1 || { tail -40 $OUT/pytest_lattice.log; exit 1; }
tail -3 $OUT/pytest_lattice.log
echo "== tiled + blosc tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_blosc.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_tiled.log 2>&1 || { tail -40 $OUT/pytest_tiled.log; exit 1; }
tail -2 $OUT/pytest_tiled.log
for i in 1 2; do
  echo "== tiled headline $i"
  timeout -k 10 300 python bench.py --tiled --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/bench_tiled_$i.json 2> $OUT/bench_tiled_$i.err || { tail -20 $OUT/bench_tiled_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_tiled_$i.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],d['config']['check'])"
  echo "== row-major headline $i"
  timeout -k 10 300 python bench.py --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/bench_rm_$i.json 2> $OUT/bench_rm_$i.err || { tail -20 $OUT/bench_rm_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_rm_$i.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['same_mix_ceiling']['frac_of_ceiling'],d['config']['check'])"
done
echo "== done"
