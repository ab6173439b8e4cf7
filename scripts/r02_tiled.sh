#!/bin/bash
# Round-2 GPU session: tiled-cascade parity, then tiled/row-major benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
echo "== tiled parity"
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiled.py -x -v --timeout 200 --timeout-method thread \
  > $OUT/pytest_tiled.log 2>&1 || { tail -40 $OUT/pytest_tiled.log; exit 1; }
tail -3 $OUT/pytest_tiled.log
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 30 --warmup 5"
for args in "" "--tiled" "--tiled --no-flags" "--workload 2048x2048_u16" "--workload 2048x2048_u16 --tiled" "--shape 5472x3648" "--shape 5472x3648 --tiled" \
            "--shape 3000x3000" "--shape 3000x3000 --tiled" "--shape 4100x4100" "--shape 4100x4100 --tiled"; do
  echo "== bench $args"
  timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print(d['value'],d['config']['batch_path'],d['config']['check'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))"
  cat $OUT/b.json >> $OUT/bench_tiled_sweep.jsonl
done

echo "== rocprof tiled headline"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_tiled -o run -- \
  python3 bench.py --tiled --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc \
  > $OUT/prof_tiled.log 2>&1 || { tail -5 $OUT/prof_tiled.log; exit 1; }
head -4 $OUT/prof_tiled/run_kernel_stats.csv | cut -c1-200
echo "== done"
