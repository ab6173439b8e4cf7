#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiled.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check --steps 30 --warmup 5"
for rep in 1 2; do
for args in "" "--tiled" "--workload 512x512_u8" "--workload 512x512_u8 --tiled" "--workload 512x512_u8 --tiled --no-flags" "--workload 2048x2048_u16 --tiled"; do
  timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { echo "FAIL $args"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$args'.ljust(36),d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))"
done
done
