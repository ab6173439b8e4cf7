#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiled.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_tiled.log 2>&1 || { tail -40 $OUT/pytest_tiled.log; exit 1; }
tail -1 $OUT/pytest_tiled.log
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check --steps 30 --warmup 5"
for rep in 1 2; do
for args in "" "--tiled" "--workload 512x512_u8" "--workload 512x512_u8 --tiled" "--workload 2048x2048_u16 --tiled" "--shape 3000x3000 --tiled" "--shape 5472x3648 --tiled"; do
  timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { echo "FAIL $args"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$args'.ljust(36),d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))" | tee -a $OUT/ab4.log
done
done
