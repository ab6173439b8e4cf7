#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 30 --warmup 5 --workload 512x512_u8"
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiled.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_tiled.log 2>&1 || { tail -40 $OUT/pytest_tiled.log; exit 1; }
tail -1 $OUT/pytest_tiled.log
for args in "" "--tiled" "--tiled --no-flags" "--chunk 256" "--chunk 256 --tiled"; do
  timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { echo "FAIL $args"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$args'.ljust(36),d['value'],d['ms_per_step'],d['config']['check'][:9],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))"
done
for args in "" "--tiled"; do
  rm -rf $OUT/kq; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kq -o run -- python3 bench.py $B --no-check $args > $OUT/kq.log 2>&1 || { tail -5 $OUT/kq.log; exit 1; }
  grep cascade_kernel $OUT/kq/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(aqz.*//' 
done
echo "== done"
